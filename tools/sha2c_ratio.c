/*
 * sha2c_ratio.c -- build-container timing harness: the reference's own
 * src/sha2.c against oracle/sha2_oracle.c (the "port" bench.py times as
 * cpu_baseline on the GPU box), on identical batches of the BASELINE
 * shapes, so the box's port figures can be read as src/sha2.c figures
 * (the port may stand in on the box only with this ratio
 * measured here).
 *
 * Built by tools/sha2c_ratio.sh into a temp directory, never into the repo
 * and never onto the GPU box: src/sha2.c is compiled where it lies in
 * /root/reference, with include/net2/sha2.h as its "sha2.h".  Context only,
 * not a parity pin -- but the digests of both are compared on every run, so
 * the two timed loops demonstrably compute the same thing.
 *
 * Each packet: Init, one Update, Final (the reference's per-payload call
 * pattern, types/signature.n2t:92, src/sign.c:298-307); threads take
 * contiguous ranges.
 *   sha2c_ratio <config c2|c3|c4> <n> <threads> <reps>
 * prints one JSON object.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "sha2.h"		/* include/net2/sha2.h: the reference's API */
#include "sha2_oracle.h"

#ifdef SHA2_UNROLL_TRANSFORM
#define FORM "unrolled"
#define ORACLE_UNROLLED 1
#else
#define FORM "rolled"
#define ORACLE_UNROLLED 0
#endif

struct batch {
	int alg;			/* 1 SHA-256, 3 SHA-512 */
	const uint8_t *base;
	uint64_t *off;
	uint32_t *len;
	size_t n;
	uint8_t *out;
	int dlen;
};

struct slice {
	const struct batch *b;
	size_t lo, hi;
	int ref;
};

static void *
run_slice(void *arg)
{
	const struct slice *s = arg;
	const struct batch *b = s->b;
	SHA2_CTX ctx;
	oracle_sha2_ctx octx;

	for (size_t i = s->lo; i < s->hi; i++) {
		const uint8_t *p = b->base + b->off[i];
		uint8_t *o = b->out + i * (size_t)b->dlen;
		if (s->ref && b->alg == 1) {
			SHA256Init(&ctx);
			SHA256Update(&ctx, p, b->len[i]);
			SHA256Final(o, &ctx);
		} else if (s->ref) {
			SHA512Init(&ctx);
			SHA512Update(&ctx, p, b->len[i]);
			SHA512Final(o, &ctx);
		} else if (b->alg == 1) {
			oracle_sha256_init(&octx);
			oracle_sha256_update(&octx, p, b->len[i]);
			oracle_sha256_final(o, &octx);
		} else {
			oracle_sha512_init(&octx);
			oracle_sha512_update(&octx, p, b->len[i]);
			oracle_sha512_final(o, &octx);
		}
	}
	return NULL;
}

static double
now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* best-of-reps wall time of the whole batch on nt threads */
static double
time_batch(const struct batch *b, int nt, int ref, int reps)
{
	pthread_t th[256];
	struct slice sl[256];
	double best = 1e30;

	for (int r = 0; r <= reps; r++) {	/* r == 0: warm-up */
		double t0 = now();
		for (int t = 0; t < nt; t++) {
			sl[t] = (struct slice){ b, b->n * t / nt, b->n * (t + 1) / nt, ref };
			pthread_create(&th[t], NULL, run_slice, &sl[t]);
		}
		for (int t = 0; t < nt; t++)
			pthread_join(th[t], NULL);
		double dt = now() - t0;
		if (r > 0 && dt < best)
			best = dt;
	}
	return best;
}

/* splitmix64, the SURVEY.md 8(d) generator */
static uint64_t
sm64(uint64_t *s)
{
	uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
	return z ^ (z >> 31);
}

int
main(int argc, char **argv)
{
	if (argc != 5) {
		fprintf(stderr, "usage: %s c2|c3|c4 n threads reps\n", argv[0]);
		return 2;
	}
	const char *cfg = argv[1];
	size_t n = strtoull(argv[2], NULL, 0);
	int nt = atoi(argv[3]), reps = atoi(argv[4]);
	if (nt < 1 || nt > 256 || n == 0)
		return 2;
	struct batch b = { 0 };
	b.alg = strcmp(cfg, "c4") == 0 ? 3 : 1;
	b.dlen = b.alg == 1 ? 32 : 64;
	b.n = n;
	b.off = malloc(n * sizeof(*b.off));
	b.len = malloc(n * sizeof(*b.len));
	uint64_t seed = strcmp(cfg, "c3") == 0 ? 3 : strcmp(cfg, "c4") == 0 ? 5 : 2;
	static const uint32_t mix[3] = { 64, 512, 1500 };
	size_t total = 0;
	for (size_t i = 0; i < n; i++) {
		b.len[i] = strcmp(cfg, "c3") == 0 ? mix[sm64(&seed) % 3] : 1024;
		b.off[i] = total;
		total += b.len[i];
	}
	uint8_t *data = malloc(total);
	for (size_t i = 0; i < total; i += 8) {
		uint64_t v = sm64(&seed);
		memcpy(data + i, &v, total - i < 8 ? total - i : 8);
	}
	b.base = data;
	uint8_t *out_ref = malloc(n * b.dlen), *out_port = malloc(n * b.dlen);

	/* the three loops alternate, best of reps each, so drift in the
	 * host's load hits all of them alike */
	double t_ref = 1e30, t_port = 1e30, t_batch = 1e30;
	int same = 1;
	for (int r = 0; r < reps; r++) {
		b.out = out_ref;
		double t = time_batch(&b, nt, 1, 1);
		t_ref = t < t_ref ? t : t_ref;
		b.out = out_port;
		t = time_batch(&b, nt, 0, 1);
		t_port = t < t_port ? t : t_port;
		same = same && memcmp(out_ref, out_port, n * b.dlen) == 0;
		/* the oracle's own batch entry (what bench.py calls), same form */
		memset(out_port, 0, n * b.dlen);
		double t0 = now();
		oracle_sha2_batch_ex(b.alg, data, b.off, b.len, 0, 0, n, out_port,
		    nt, ORACLE_UNROLLED);
		t = now() - t0;
		t_batch = t < t_batch ? t : t_batch;
		same = same && memcmp(out_ref, out_port, n * b.dlen) == 0;
	}
	printf("{\"config\": \"%s\", \"form\": \"%s\", \"n\": %zu, \"threads\": %d, "
	    "\"ref_sha2c_digests_per_s\": %.1f, \"port_digests_per_s\": %.1f, "
	    "\"port_batch_digests_per_s\": %.1f, \"port_over_ref\": %.4f, "
	    "\"port_batch_over_ref\": %.4f, \"digests_identical\": %s}\n",
	    cfg, FORM, n, nt, n / t_ref, n / t_port, n / t_batch, t_ref / t_port,
	    t_ref / t_batch, same ? "true" : "false");
	return same ? 0 : 1;
}
