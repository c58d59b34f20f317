/*
 * test_sign.c -- C-level test of the signed-payload path over the MI355X
 * hash ABI.  Part 1 restates the reference's test/sign.c:57-185 (P-521 key
 * pair from test/sign.c:27-45): sign a maxmsglen message, validate it, a
 * second signature differs, a tampered message is invalid, pubkey(priv) ==
 * pubkey(pub).  Part 2 checks the hash-then-sign objects of
 * types/signature.n2t and their batched forms: every digest the GPU feeds to
 * ECDSA is checked independently by verifying the signature against an
 * OpenSSL-computed digest of the same payload (OpenSSL here is the test's
 * independent reference, never the product path).
 *
 * Usage: test_sign <priv.pem> <pub.pem> [all|cpu]; exit 0 = pass.  "all"
 * (default) needs a GPU; "cpu" runs only part 1, which hashes nothing.
 */
#include "../../include/net2/hash.h"
#include "../../include/net2/sign.h"
#include "../../include/net2/signature.h"
#include "../../include/net2/signed_carver.h"

#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

#include <openssl/evp.h>
#include <openssl/pem.h>

static int failures;

#define CHECK(cond) do {							\
	if (!(cond)) {							\
		fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__,	\
		    #cond);						\
		failures++;						\
	}								\
} while (0)

static char *
slurp(const char *path, size_t *len)
{
	FILE *f = fopen(path, "rb");
	char *buf;
	long n;

	if (f == NULL)
		return NULL;
	fseek(f, 0, SEEK_END);
	n = ftell(f);
	fseek(f, 0, SEEK_SET);
	buf = malloc((size_t)n + 1);
	if (buf == NULL || fread(buf, 1, (size_t)n, f) != (size_t)n) {
		fclose(f);
		free(buf);
		return NULL;
	}
	fclose(f);
	buf[n] = 0;
	*len = (size_t)n;
	return buf;
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;

static uint8_t
rnd8(void)
{
	rng_state ^= rng_state << 13;
	rng_state ^= rng_state >> 7;
	rng_state ^= rng_state << 17;
	return (uint8_t)rng_state;
}

/* Independent reference digest (OpenSSL EVP), test-only. */
static void
ref_digest(int alg, const uint8_t *m, size_t len, uint8_t *out)
{
	const EVP_MD *md = alg == 1 ? EVP_sha256() : alg == 2 ? EVP_sha384()
	    : EVP_sha512();
	unsigned int ol = 0;

	EVP_Digest(m, len, out, &ol, md, NULL);
}

static int
ref_verify(EVP_PKEY *pub, const uint8_t *sig, size_t siglen,
    const uint8_t *dig, size_t dlen)
{
	EVP_PKEY_CTX *pc = EVP_PKEY_CTX_new(pub, NULL);
	int ok = pc && EVP_PKEY_verify_init(pc) == 1 &&
	    EVP_PKEY_verify(pc, sig, siglen, dig, dlen) == 1;

	EVP_PKEY_CTX_free(pc);
	return ok;
}

/* Part 1: test/sign.c restated. */
static void
test_reference_flow(struct net2x_sign_ctx *priv, struct net2x_sign_ctx *pub)
{
	size_t maxlen = net2x_signctx_maxmsglen(priv);
	uint8_t *msg = malloc(maxlen), *sig = malloc(maxlen),
	    *sig2 = malloc(maxlen);
	size_t siglen = maxlen, sig2len = maxlen;
	uint8_t pk1[256], pk2[256];
	size_t pk1len = sizeof(pk1), pk2len = sizeof(pk2);

	CHECK(maxlen > 0);
	for (size_t i = 0; i < maxlen; i++)
		msg[i] = rnd8();
	CHECK(net2x_signctx_sign(priv, msg, maxlen, sig, &siglen) == 0);
	CHECK(net2x_signctx_validate(pub, sig, siglen, msg, maxlen) == 1);
	/* a second signature of the same message differs (random k) */
	CHECK(net2x_signctx_sign(priv, msg, maxlen, sig2, &sig2len) == 0);
	CHECK(siglen != sig2len || memcmp(sig, sig2, siglen) != 0);
	CHECK(net2x_signctx_validate(pub, sig2, sig2len, msg, maxlen) == 1);
	/* tampered message is invalid (test/sign.c:129-148) */
	msg[0] ^= 0xff;
	msg[1] ^= 0x5a;
	CHECK(net2x_signctx_validate(pub, sig, siglen, msg, maxlen) == 0);
	/* a public context cannot sign */
	CHECK(net2x_signctx_sign(pub, msg, maxlen, sig2, &sig2len) == EINVAL);
	/* public keys agree (test/sign.c:151-180) */
	CHECK(net2x_signctx_pubkey(priv, pk1, &pk1len) == 0);
	CHECK(net2x_signctx_pubkey(pub, pk2, &pk2len) == 0);
	CHECK(pk1len == pk2len && memcmp(pk1, pk2, pk1len) == 0);
	CHECK(pk1len == 133 && pk1[0] == 0x04);	/* uncompressed P-521 */
	CHECK(strcmp(net2x_signctx_name(priv), "ecdsa") == 0);
	CHECK(net2x_sign_findname("ecdsa") == 0 && net2x_sign_getname(1) == NULL);
	free(msg);
	free(sig);
	free(sig2);
}

/* Fingerprint = SHA-256 of the uncompressed point (src/sign.c:258-320). */
static void
test_fingerprint(struct net2x_sign_ctx *priv, struct net2x_sign_ctx *pub)
{
	uint8_t fp1[32], fp2[32], want[32], pk[256];
	size_t pklen = sizeof(pk);
	struct net2x_sign_ctx *clone;

	CHECK(net2x_signctx_fingerprint(priv, fp1) == 0);
	CHECK(net2x_signctx_fingerprint(pub, fp2) == 0);
	CHECK(memcmp(fp1, fp2, 32) == 0);
	CHECK(net2x_signctx_pubkey(pub, pk, &pklen) == 0);
	ref_digest(1, pk, pklen, want);
	CHECK(memcmp(fp1, want, 32) == 0);
	clone = net2x_signctx_clone(pub);
	CHECK(clone != NULL);
	CHECK(net2x_signctx_fingerprint(clone, fp2) == 0 &&
	    memcmp(fp2, want, 32) == 0);
	net2x_signctx_free(clone);
}

/* Part 2: signature objects, single and batched. */
static void
test_signatures(struct net2x_sign_ctx *priv, struct net2x_sign_ctx *pub,
    EVP_PKEY *refpub)
{
	enum { N = 1000 };
	static const uint32_t shapes[] = { 0, 1, 64, 111, 112, 512, 1024, 1500,
	    65536 };
	uint64_t offs[N];
	uint32_t lens[N];
	size_t total = 0;
	uint8_t *buf, dig[64];
	struct net2x_signature one, *many;
	struct iovec iov[3];
	int valid, *vv;

	for (int i = 0; i < N; i++) {
		lens[i] = shapes[i % 9] == 65536 && i > 9 ? 777 : shapes[i % 9];
		offs[i] = total;
		total += lens[i] + (i & 3);	/* ragged, unaligned */
	}
	buf = malloc(total + 1);
	for (size_t i = 0; i < total; i++)
		buf[i] = rnd8();

	/* single, scattered over three iovecs (signature.n2t:60-119) */
	iov[0].iov_base = buf;
	iov[0].iov_len = 100;
	iov[1].iov_base = buf + 100;
	iov[1].iov_len = 0;
	iov[2].iov_base = buf + 100;
	iov[2].iov_len = 1400;
	for (int alg = 1; alg <= 3; alg++) {
		CHECK(net2x_signature_create(&one, iov, 3, alg, priv) == 0);
		CHECK(strcmp(one.hash_alg, net2_hash_getname(alg)) == 0);
		CHECK(strcmp(one.sign_alg, "ecdsa") == 0);
		CHECK(net2x_signature_validate(&one, iov, 3, pub, &valid) == 0 &&
		    valid == 1);
		ref_digest(alg, buf, 1500, dig);
		CHECK(ref_verify(refpub, one.data, one.datalen, dig,
		    (size_t)net2_hash_gethashlen(alg)));
		buf[700] ^= 1;				/* tamper */
		CHECK(net2x_signature_validate(&one, iov, 3, pub, &valid) == 0 &&
		    valid == 0);
		buf[700] ^= 1;
		net2x_signature_deinit(&one);
	}
	/* error behaviour of signature.n2t:69-72, 133-158 */
	CHECK(net2x_signature_create(&one, iov, 3, 0, priv) == EINVAL);
	CHECK(net2x_signature_create(&one, iov, 3, 4, priv) == EINVAL);
	CHECK(net2x_signature_create(&one, iov, 3, 99, priv) == EINVAL);
	CHECK(net2x_signature_create(&one, iov, 3, 3, priv) == 0);
	free(one.hash_alg);
	one.hash_alg = strdup("MD5");
	CHECK(net2x_signature_validate(&one, iov, 3, pub, &valid) == EOPNOTSUPP &&
	    valid == 0);
	free(one.hash_alg);
	one.hash_alg = strdup("SHA512");
	free(one.sign_alg);
	one.sign_alg = strdup("rsa");
	CHECK(net2x_signature_validate(&one, iov, 3, pub, &valid) == EINVAL);
	net2x_signature_deinit(&one);
	CHECK(net2x_signature_validate(NULL, iov, 3, pub, &valid) == EINVAL);

	/* batched: one GPU hash launch for all N payloads, then ECDSA */
	many = calloc(N, sizeof(*many));
	vv = calloc(N, sizeof(*vv));
	CHECK(net2x_signature_create_batch(many, buf, offs, lens, N, 3, priv,
	    8) == 0);
	for (int i = 0; i < N; i += 37) {
		ref_digest(3, buf + offs[i], lens[i], dig);
		CHECK(ref_verify(refpub, many[i].data, many[i].datalen, dig, 64));
	}
	CHECK(net2x_signature_validate_batch(many, buf, offs, lens, N, pub, vv,
	    8) == 0);
	for (int i = 0; i < N; i++)
		CHECK(vv[i] == 1);
	/* mixed hash algorithms and broken entries in one validate batch */
	net2x_signature_deinit(&many[5]);
	CHECK(net2x_signature_create(&many[5], &(struct iovec){ buf + offs[5],
	    lens[5] }, 1, 1, priv) == 0);		/* SHA256 entry */
	free(many[6].hash_alg);
	many[6].hash_alg = strdup("MD5");		/* unknown hash */
	buf[offs[7]] ^= 0x80;				/* tampered payload */
	CHECK(lens[7] > 0);
	CHECK(net2x_signature_validate_batch(many, buf, offs, lens, N, pub, vv,
	    4) == 0);
	for (int i = 0; i < N; i++)
		CHECK(vv[i] == (i == 6 || i == 7 ? 0 : 1));
	for (int i = 0; i < N; i++)
		net2x_signature_deinit(&many[i]);
	free(many);
	free(vv);
	free(buf);
}

/*
 * Part 3: the signed carver's signature step batched per tick
 * (net2/signed_carver.h) at BASELINE configs[0]'s shape, 4096 x 1 KiB
 * payloads: carvers with two sign contexts each (src/signed_carver.c:
 * 407-432), added from four threads, one tick; then the combiner checks
 * (:265-338) of every signature, with tampered payloads, an unknown hash
 * name and a wrong sign algorithm among them, in one more tick.
 */
struct adder {
	struct net2_sc_collector	*c;
	struct net2_sc_sign_req		*reqs;
	size_t				 lo, hi;
};

static void *
add_some(void *arg)
{
	struct adder *a = arg;

	for (size_t i = a->lo; i < a->hi; i++)
		CHECK(net2_sc_collector_add_sign(a->c, &a->reqs[i]) == 0);
	return NULL;
}

static double
now_s(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void
test_carver_tick(struct net2x_sign_ctx *priv, struct net2x_sign_ctx *pub,
    EVP_PKEY *refpub)
{
	enum { N = 4096, L = 1024, NS = 2 };
	uint8_t *buf = malloc((size_t)N * L), dig[64];
	struct iovec *iov = calloc(2 * N, sizeof(*iov));
	struct net2_sc_sign_req *reqs = calloc(N, sizeof(*reqs));
	struct net2x_signature *sigs = calloc((size_t)N * NS, sizeof(*sigs));
	struct net2_sc_validate_req *vr = calloc((size_t)N * NS, sizeof(*vr));
	struct net2x_sign_ctx *ctxs[NS] = { priv, net2x_signctx_clone(priv) };
	struct net2_sc_collector *c = net2_sc_collector_new(8);
	struct adder ad[4];
	pthread_t tid[4];
	size_t ns = 0, nv = 0;
	double t0, t_sign, t_val;
	int bad = 0;

	CHECK(c != NULL && ctxs[1] != NULL);
	for (size_t i = 0; i < (size_t)N * L; i++)
		buf[i] = rnd8();
	for (int i = 0; i < N; i++) {
		/* most payloads one segment, every 5th split in two */
		iov[2 * i].iov_base = buf + (size_t)i * L;
		iov[2 * i].iov_len = i % 5 ? L : 300;
		iov[2 * i + 1].iov_base = buf + (size_t)i * L + 300;
		iov[2 * i + 1].iov_len = L - 300;
		reqs[i].payload = &iov[2 * i];
		reqs[i].iovcnt = i % 5 ? 1 : 2;
		reqs[i].hash_alg = i % 3 ? 3 : 1;	/* SHA512, some SHA256 */
		reqs[i].num_signatures = NS;
		reqs[i].signatures = ctxs;
		reqs[i].out = &sigs[(size_t)i * NS];
	}
	reqs[N - 1].hash_alg = 4;	/* keyed row: not a sighash -> EINVAL */
	for (int t = 0; t < 4; t++) {
		ad[t] = (struct adder){ c, reqs, (size_t)N * t / 4,
		    (size_t)N * (t + 1) / 4 };
		pthread_create(&tid[t], NULL, add_some, &ad[t]);
	}
	for (int t = 0; t < 4; t++)
		pthread_join(tid[t], NULL);
	t0 = now_s();
	CHECK(net2_sc_collector_tick(c, NULL, &ns, &nv) == 0);
	t_sign = now_s() - t0;
	CHECK(ns == N && nv == 0);
	CHECK(reqs[N - 1].rc == EINVAL);
	for (int i = 0; i < N - 1; i++) {
		CHECK(reqs[i].rc == 0);
		if (i % 97 != 0)
			continue;
		for (int k = 0; k < NS; k++) {
			struct net2x_signature *sg = &sigs[(size_t)i * NS + k];
			ref_digest(reqs[i].hash_alg, buf + (size_t)i * L, L, dig);
			CHECK(strcmp(sg->hash_alg,
			    net2_hash_getname(reqs[i].hash_alg)) == 0);
			CHECK(ref_verify(refpub, sg->data, sg->datalen, dig,
			    (size_t)net2_hash_gethashlen(reqs[i].hash_alg)));
		}
	}
	/* checks of every signature, some broken */
	for (int i = 0; i < N - 1; i++)
		for (int k = 0; k < NS; k++) {
			struct net2_sc_validate_req *q = &vr[(size_t)i * NS + k];
			q->payload = reqs[i].payload;
			q->iovcnt = reqs[i].iovcnt;
			q->sig = &sigs[(size_t)i * NS + k];
			q->sctx = pub;
			q->result = -1;
			CHECK(net2_sc_collector_add_validate(c, q) == 0);
		}
	for (int i = 10; i < N - 1; i += 211)
		buf[(size_t)i * L + 700] ^= 0x01;	/* tampered payload */
	free(sigs[2 * 3].hash_alg);
	sigs[2 * 3].hash_alg = strdup("MD5");		/* unknown hash */
	free(sigs[2 * 4 + 1].sign_alg);
	sigs[2 * 4 + 1].sign_alg = strdup("rsa");	/* wrong sign alg */
	t0 = now_s();
	CHECK(net2_sc_collector_tick(c, NULL, &ns, &nv) == 0);
	t_val = now_s() - t0;
	CHECK(ns == 0 && nv == (size_t)(N - 1) * NS);
	for (int i = 0; i < N - 1; i++)
		for (int k = 0; k < NS; k++) {
			const int r = vr[(size_t)i * NS + k].result;
			int want = 0;
			if (i >= 10 && (i - 10) % 211 == 0)
				want = EINVAL;
			if ((i == 3 && k == 0) || (i == 4 && k == 1))
				want = EIO;
			if (r != want)
				bad++;
		}
	CHECK(bad == 0);
	/* an empty tick is a no-op */
	CHECK(net2_sc_collector_tick(c, NULL, &ns, &nv) == 0 && ns == 0 && nv == 0);
	printf("carver tick: %d carvers x %d signatures: sign %.1f ms, "
	    "validate %.1f ms\n", N, NS, t_sign * 1e3, t_val * 1e3);
	for (size_t i = 0; i < (size_t)N * NS; i++)
		net2x_signature_deinit(&sigs[i]);
	net2_sc_collector_free(c);
	net2x_signctx_free(ctxs[1]);
	free(buf);
	free(iov);
	free(reqs);
	free(sigs);
	free(vr);
}

/*
 * Part 4: the hash-only tick (net2_sc_hash_req), bound as the reference's
 * signed_carver.c would bind it: the callback
 * gets the digest and signs it with a sign context the tick knows nothing
 * about -- here this repository's net2x_signctx_sign stands in for the
 * reference's src/sign.c net2_signctx_sign (same ECDSA over the digest,
 * src/sign.c:478-516).  4096 x 1 KiB payloads (BASELINE configs[0]), mixed
 * SHA-256 / 384 / 512, some split over two iovecs, added from four
 * threads; every digest is compared with OpenSSL's, every callback must run
 * exactly once, and the signatures verify.  Then the validate side
 * (signctx_validate, :265-338): digest in the callback, the signature
 * checked there, tampered payloads found.
 */
struct hjob {
	struct net2_sc_hash_req	 h;
	struct net2x_sign_ctx	*ctx;		/* sign or validate with */
	const uint8_t		*sig;		/* validate: the signature */
	size_t			 siglen;
	uint8_t			 out[160];	/* sign: the signature */
	size_t			 outlen;
	int			 calls, verdict;
	pthread_t		 thread;
};

static void
hjob_sign(struct net2_sc_hash_req *h, void *arg)
{
	struct hjob *j = arg;

	CHECK(&j->h == h);
	__atomic_add_fetch(&j->calls, 1, __ATOMIC_RELAXED);
	j->thread = pthread_self();
	j->outlen = sizeof(j->out);
	j->verdict = h->rc == 0 ? net2x_signctx_sign(j->ctx, h->digest,
	    h->digestlen, j->out, &j->outlen) : h->rc;
}

static void
hjob_validate(struct net2_sc_hash_req *h, void *arg)
{
	struct hjob *j = arg;

	__atomic_add_fetch(&j->calls, 1, __ATOMIC_RELAXED);
	j->thread = pthread_self();
	/* signature.n2t:160-161 after its hashbuf; finok / EINVAL / EIO as
	 * signed_carver.c:316-319,333-336 */
	j->verdict = h->rc != 0 ? EIO : net2x_signctx_validate(j->ctx, j->sig,
	    j->siglen, h->digest, h->digestlen) == 1 ? 0 : EINVAL;
}

struct hadder {
	struct net2_sc_collector	*c;
	struct hjob			*jobs;
	size_t				 lo, hi;
};

static void *
hadd_some(void *arg)
{
	struct hadder *a = arg;

	for (size_t i = a->lo; i < a->hi; i++)
		CHECK(net2_sc_collector_add_hash(a->c, &a->jobs[i].h) == 0);
	return NULL;
}

static void
test_hash_tick(struct net2x_sign_ctx *priv, struct net2x_sign_ctx *pub,
    EVP_PKEY *refpub)
{
	enum { N = 4096, L = 1024 };
	uint8_t *buf = malloc((size_t)N * L), dig[64];
	struct iovec *iov = calloc(2 * N, sizeof(*iov));
	struct hjob *jobs = calloc(N, sizeof(*jobs));
	struct hjob *vj = calloc(N, sizeof(*vj));
	struct net2_sc_collector *c = net2_sc_collector_new(8);
	struct hadder ad[4];
	pthread_t tid[4];
	size_t nh = 0, ns = 0, nv = 0;
	int bad_digest = 0, bad_calls = 0, bad_sig = 0, bad_val = 0, other = 0;
	double t0, t_sign, t_val;

	CHECK(c != NULL);
	for (size_t i = 0; i < (size_t)N * L; i++)
		buf[i] = rnd8();
	for (int i = 0; i < N; i++) {
		iov[2 * i].iov_base = buf + (size_t)i * L;
		iov[2 * i].iov_len = i % 7 ? L : 333;
		iov[2 * i + 1].iov_base = buf + (size_t)i * L + 333;
		iov[2 * i + 1].iov_len = L - 333;
		jobs[i].h.payload = &iov[2 * i];
		jobs[i].h.iovcnt = i % 7 ? 1 : 2;
		jobs[i].h.hash_alg = 1 + i % 3;
		jobs[i].h.done = hjob_sign;
		jobs[i].h.arg = &jobs[i];
		jobs[i].ctx = priv;
	}
	jobs[N - 1].h.hash_alg = 6;	/* keyed row: EINVAL, callback still runs */
	for (int t = 0; t < 4; t++) {
		ad[t] = (struct hadder){ c, jobs, (size_t)N * t / 4,
		    (size_t)N * (t + 1) / 4 };
		pthread_create(&tid[t], NULL, hadd_some, &ad[t]);
	}
	for (int t = 0; t < 4; t++)
		pthread_join(tid[t], NULL);
	t0 = now_s();
	CHECK(net2_sc_collector_tick(c, &nh, &ns, &nv) == 0);
	t_sign = now_s() - t0;
	CHECK(nh == N && ns == 0 && nv == 0);
	CHECK(jobs[N - 1].h.rc == EINVAL && jobs[N - 1].calls == 1 &&
	    jobs[N - 1].verdict == EINVAL);
	for (int i = 0; i < N - 1; i++) {
		const int alg = jobs[i].h.hash_alg;
		if (jobs[i].calls != 1)
			bad_calls++;
		ref_digest(alg, buf + (size_t)i * L, L, dig);
		if (jobs[i].h.rc != 0 || jobs[i].h.digestlen !=
		    (uint32_t)net2_hash_gethashlen(alg) ||
		    memcmp(jobs[i].h.digest, dig, jobs[i].h.digestlen) != 0)
			bad_digest++;
		if (jobs[i].verdict != 0 || (i % 61 == 0 && !ref_verify(refpub,
		    jobs[i].out, jobs[i].outlen, dig, jobs[i].h.digestlen)))
			bad_sig++;
		if (!pthread_equal(jobs[i].thread, jobs[0].thread))
			other++;
	}
	CHECK(bad_calls == 0);
	CHECK(bad_digest == 0);
	CHECK(bad_sig == 0);
	CHECK(other > 0);	/* the callbacks ran on more than one thread */
	/* the validate side, some payloads tampered, in place (no collector) */
	for (int i = 0; i < N - 1; i++) {
		vj[i].h = jobs[i].h;
		vj[i].h.done = hjob_validate;
		vj[i].h.arg = &vj[i];
		vj[i].ctx = pub;
		vj[i].sig = jobs[i].out;
		vj[i].siglen = jobs[i].outlen;
	}
	for (int i = 5; i < N - 1; i += 101)
		buf[(size_t)i * L + 900] ^= 0x40;
	{
		struct net2_sc_hash_req *hr = calloc(N - 1, sizeof(*hr));
		/* net2_sc_hash_tick works on an array: copy, tick, then check
		 * that each callback got its own element */
		for (int i = 0; i < N - 1; i++) {
			hr[i] = vj[i].h;
		}
		t0 = now_s();
		CHECK(net2_sc_hash_tick(hr, N - 1, 8) == 0);
		t_val = now_s() - t0;
		for (int i = 0; i < N - 1; i++) {
			const int want = i >= 5 && (i - 5) % 101 == 0 ? EINVAL : 0;
			if (vj[i].calls != 1 || vj[i].verdict != want)
				bad_val++;
		}
		free(hr);
	}
	CHECK(bad_val == 0);
	/* an empty tick is a no-op; a bad argument is EINVAL */
	CHECK(net2_sc_collector_tick(c, &nh, &ns, &nv) == 0 && nh == 0);
	CHECK(net2_sc_hash_tick(NULL, 1, 1) == EINVAL);
	CHECK(net2_sc_hash_tick(NULL, 0, 1) == 0);
	printf("hash tick: %d payloads, callbacks sign: %.1f ms, validate "
	    "%.1f ms\n", N, t_sign * 1e3, t_val * 1e3);
	net2_sc_collector_free(c);
	free(buf);
	free(iov);
	free(jobs);
	free(vj);
}

int
main(int argc, char **argv)
{
	char *privpem, *pubpem;
	size_t privlen, publen;
	struct net2x_sign_ctx *priv, *pub;
	EVP_PKEY *refpub;
	BIO *bio;
	int ndev = 0;

	int cpu_only = argc == 4 && strcmp(argv[3], "cpu") == 0;

	if (argc != 3 && argc != 4) {
		fprintf(stderr, "usage: %s priv.pem pub.pem [all|cpu]\n", argv[0]);
		return 2;
	}
	if (!cpu_only && (net2_sha2_device_count(&ndev) != 0 || ndev < 1)) {
		fprintf(stderr, "no gfx950 device\n");
		return 3;
	}
	privpem = slurp(argv[1], &privlen);
	pubpem = slurp(argv[2], &publen);
	if (privpem == NULL || pubpem == NULL)
		return 2;
	/* test/sign.c:66,69 */
	priv = net2x_signctx_privnew(net2x_sign_ecdsa, privpem, privlen);
	pub = net2x_signctx_pubnew(net2x_sign_ecdsa, pubpem, publen);
	CHECK(priv != NULL && pub != NULL);
	CHECK(net2x_signctx_pubnew(1, pubpem, publen) == NULL);	/* bad alg */
	CHECK(net2x_signctx_privnew(0, pubpem, publen) == NULL);	/* not priv */
	bio = BIO_new_mem_buf(pubpem, (int)publen);
	refpub = PEM_read_bio_PUBKEY(bio, NULL, NULL, NULL);
	BIO_free(bio);
	if (priv && pub && refpub) {
		test_reference_flow(priv, pub);
		if (!cpu_only) {
			test_fingerprint(priv, pub);
			test_signatures(priv, pub, refpub);
			test_carver_tick(priv, pub, refpub);
			test_hash_tick(priv, pub, refpub);
		}
	}
	EVP_PKEY_free(refpub);
	net2x_signctx_free(priv);
	net2x_signctx_free(pub);
	free(privpem);
	free(pubpem);
	printf("%s%s (%d failures)\n", failures ? "FAIL" : "PASS",
	    cpu_only ? " cpu-only" : "", failures);
	return failures ? 1 : 0;
}
