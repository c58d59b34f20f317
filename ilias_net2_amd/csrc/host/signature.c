/*
 * signature.c -- hash-then-sign objects (types/signature.n2t:60-189)
 * restated over iovecs, and their batched forms for the signed carver
 * (src/signed_carver.c:407-432 creates one signature per sign context over
 * the whole payload; :265-338 validates one per received payload).
 *
 * The digest of every payload comes from the MI355X path
 * (net2_hashctx_hashiov for one payload, net2_sha2_batch for a batch); the
 * ECDSA step stays on the host (OpenSSL), spread over a few threads in the
 * batched forms.
 */
#include "../../../include/net2/signature.h"
#include "../../../include/net2/hash.h"
#include "signature_int.h"

#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define NET2_EXPORT __attribute__((visibility("default")))

static char *
dupstr(const char *s)
{
	size_t n = strlen(s) + 1;
	char *d = malloc(n);

	if (d != NULL)
		memcpy(d, s, n);
	return d;
}

NET2_EXPORT void
net2x_signature_deinit(struct net2x_signature *s)
{
	if (s == NULL)
		return;
	free(s->sign_alg);
	free(s->hash_alg);
	free(s->data);
	s->sign_alg = s->hash_alg = NULL;
	s->data = NULL;
	s->datalen = 0;
}

/* Fill s from an already computed digest (signature.n2t:74-100); shared
 * with the tick-batched carver step (signed_carver.c), hidden. */
int
sign_digest(struct net2x_signature *s, const uint8_t *digest, size_t dlen,
    const char *hash_name, struct net2x_sign_ctx *sign)
{
	size_t cap = net2x_signctx_maxmsglen(sign);
	int rc;

	memset(s, 0, sizeof(*s));
	if ((s->sign_alg = dupstr(net2x_signctx_name(sign))) == NULL ||
	    (s->hash_alg = dupstr(hash_name)) == NULL ||
	    (s->data = malloc(cap ? cap : 1)) == NULL) {
		net2x_signature_deinit(s);
		return ENOMEM;
	}
	s->datalen = cap;
	if ((rc = net2x_signctx_sign(sign, digest, dlen, s->data,
	    &s->datalen)) != 0) {
		net2x_signature_deinit(s);
		return rc;
	}
	return 0;
}

NET2_EXPORT int
net2x_signature_create(struct net2x_signature *s, const struct iovec *to_sign,
    size_t iovcnt, int hash_alg, struct net2x_sign_ctx *sign)
{
	const char *hash_name;
	uint8_t digest[64];
	int hl, rc;

	if (s == NULL || (to_sign == NULL && iovcnt > 0) || sign == NULL)
		return EINVAL;
	if ((hash_name = net2_hash_getname(hash_alg)) == NULL)
		return EINVAL;
	if ((hl = net2_hash_gethashlen(hash_alg)) <= 0 ||
	    net2_hash_getkeylen(hash_alg) != 0)
		return EINVAL;		/* sighash rows are unkeyed SHA-2 */
	if ((rc = net2_hashctx_hashiov(hash_alg, NULL, 0, to_sign, iovcnt,
	    digest, sizeof(digest))) != 0)
		return rc == EINVAL ? EINVAL : ENOMEM;	/* signature.n2t:93-95 */
	return sign_digest(s, digest, (size_t)hl, hash_name, sign);
}

/* signature.n2t:133-141 argument checks; returns the hash row or -errno. */
static int
validate_prologue(const struct net2x_signature *s, int *valid)
{
	int alg;

	if (valid == NULL)
		return -EINVAL;
	*valid = 0;			/* default to invalid, to be safe */
	if (s == NULL || s->data == NULL || s->hash_alg == NULL ||
	    s->sign_alg == NULL)
		return -EINVAL;
	if ((alg = net2_hash_findname(s->hash_alg)) == -1)
		return -EOPNOTSUPP;
	if (net2_hash_getkeylen(alg) != 0 || net2_hash_gethashlen(alg) <= 0)
		return -EOPNOTSUPP;
	return alg;
}

NET2_EXPORT int
net2x_signature_validate(const struct net2x_signature *s,
    const struct iovec *to_sign, size_t iovcnt, struct net2x_sign_ctx *sign,
    int *valid)
{
	uint8_t digest[64];
	int alg, rc;

	if ((alg = validate_prologue(s, valid)) < 0)
		return -alg;
	if ((to_sign == NULL && iovcnt > 0) || sign == NULL)
		return EINVAL;
	if ((rc = net2_hashctx_hashiov(alg, NULL, 0, to_sign, iovcnt, digest,
	    sizeof(digest))) != 0)
		return ENOMEM;				/* signature.n2t:148-151 */
	if (strcmp(net2x_signctx_name(sign), s->sign_alg) != 0)
		return EINVAL;				/* signature.n2t:155-158 */
	*valid = net2x_signctx_validate(sign, s->data, s->datalen, digest,
	    (size_t)net2_hash_gethashlen(alg));
	return 0;
}

/* ---- batched forms -------------------------------------------------- */

struct ecdsa_job {
	int			 create;
	size_t			 lo, hi;
	const uint8_t		*digests;
	size_t			 dlen;
	const char		*hash_name;
	struct net2x_sign_ctx	*sign;
	struct net2x_signature	*out;		/* create */
	const struct net2x_signature *sigs;	/* validate */
	const int		*alg_of;	/* validate: hash row or -errno */
	const size_t		*dig_at;	/* validate: digest offset */
	int			*valid;
	int			 rc;
};

static void *
ecdsa_worker(void *arg)
{
	struct ecdsa_job *j = arg;

	for (size_t i = j->lo; i < j->hi && j->rc == 0; i++) {
		if (j->create) {
			j->rc = sign_digest(&j->out[i], j->digests + i * j->dlen,
			    j->dlen, j->hash_name, j->sign);
			continue;
		}
		if (j->alg_of[i] < 0 ||
		    strcmp(net2x_signctx_name(j->sign), j->sigs[i].sign_alg) != 0)
			continue;	/* valid[i] stays 0 */
		j->valid[i] = net2x_signctx_validate(j->sign, j->sigs[i].data,
		    j->sigs[i].datalen, j->digests + j->dig_at[i],
		    (size_t)net2_hash_gethashlen(j->alg_of[i]));
	}
	return NULL;
}

static int
run_ecdsa(struct ecdsa_job *proto, size_t n, int nthreads)
{
	struct ecdsa_job jobs[64];
	pthread_t tid[64];
	int t, started, rc = 0;

	if (nthreads <= 0) {
		long c = sysconf(_SC_NPROCESSORS_ONLN);
		nthreads = c > 0 ? (int)c : 1;
	}
	if (nthreads > 64)
		nthreads = 64;
	if ((size_t)nthreads > n)
		nthreads = n ? (int)n : 1;
	for (t = 0; t < nthreads; t++) {
		jobs[t] = *proto;
		jobs[t].lo = n * t / nthreads;
		jobs[t].hi = n * (t + 1) / nthreads;
	}
	for (started = 1; started < nthreads; started++)
		if (pthread_create(&tid[started], NULL, ecdsa_worker,
		    &jobs[started]) != 0)
			break;
	ecdsa_worker(&jobs[0]);
	for (t = started; t < nthreads; t++)	/* threads we could not start */
		ecdsa_worker(&jobs[t]);
	for (t = 1; t < started; t++)
		pthread_join(tid[t], NULL);
	for (t = 0; t < nthreads; t++)
		if (jobs[t].rc != 0 && rc == 0)
			rc = jobs[t].rc;
	return rc;
}

NET2_EXPORT int
net2x_signature_create_batch(struct net2x_signature *out, const uint8_t *base,
    const uint64_t *offsets, const uint32_t *lens, size_t n, int hash_alg,
    struct net2x_sign_ctx *sign, int nthreads)
{
	struct ecdsa_job job;
	const char *hash_name;
	uint8_t *digests;
	int hl, rc;

	if (n == 0)
		return 0;
	if (out == NULL || offsets == NULL || lens == NULL || sign == NULL)
		return EINVAL;
	if ((hash_name = net2_hash_getname(hash_alg)) == NULL ||
	    (hl = net2_hash_gethashlen(hash_alg)) <= 0 ||
	    net2_hash_getkeylen(hash_alg) != 0)
		return EINVAL;
	if ((digests = malloc(n * (size_t)hl)) == NULL)
		return ENOMEM;
	/* one GPU batch for every payload's digest */
	rc = net2_sha2_batch(hash_alg, base, offsets, lens, 0, 0, n, digests,
	    0);
	if (rc == 0) {
		memset(out, 0, n * sizeof(*out));
		memset(&job, 0, sizeof(job));
		job.create = 1;
		job.digests = digests;
		job.dlen = (size_t)hl;
		job.hash_name = hash_name;
		job.sign = sign;
		job.out = out;
		rc = run_ecdsa(&job, n, nthreads);
		if (rc != 0)
			for (size_t i = 0; i < n; i++)
				net2x_signature_deinit(&out[i]);
	}
	free(digests);
	return rc;
}

NET2_EXPORT int
net2x_signature_validate_batch(const struct net2x_signature *sigs,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lens,
    size_t n, struct net2x_sign_ctx *sign, int *valid, int nthreads)
{
	struct ecdsa_job job;
	int *alg_of = NULL;
	size_t *dig_at = NULL, *idx = NULL;
	uint64_t *sub_off = NULL;
	uint32_t *sub_len = NULL;
	uint8_t *digests = NULL, *sub_dig = NULL;
	int rc = 0;

	if (n == 0)
		return 0;
	if (sigs == NULL || offsets == NULL || lens == NULL || sign == NULL ||
	    valid == NULL)
		return EINVAL;
	alg_of = malloc(n * sizeof(*alg_of));
	dig_at = malloc(n * sizeof(*dig_at));
	idx = malloc(n * sizeof(*idx));
	sub_off = malloc(n * sizeof(*sub_off));
	sub_len = malloc(n * sizeof(*sub_len));
	digests = malloc(n * 64);
	sub_dig = malloc(n * 64);
	if (!alg_of || !dig_at || !idx || !sub_off || !sub_len || !digests ||
	    !sub_dig) {
		rc = ENOMEM;
		goto out;
	}
	for (size_t i = 0; i < n; i++) {
		int v;
		alg_of[i] = validate_prologue(&sigs[i], &v);
		valid[i] = 0;
		dig_at[i] = i * 64;
	}
	/* one GPU batch per hash algorithm named by the signatures */
	for (int alg = 1; alg < net2_hashmax && rc == 0; alg++) {
		size_t m = 0;
		int hl = net2_hash_gethashlen(alg);
		for (size_t i = 0; i < n; i++)
			if (alg_of[i] == alg) {
				idx[m] = i;
				sub_off[m] = offsets[i];
				sub_len[m] = lens[i];
				m++;
			}
		if (m == 0)
			continue;
		rc = net2_sha2_batch(alg, base, sub_off, sub_len, 0, 0, m,
		    sub_dig, 0);
		for (size_t k = 0; rc == 0 && k < m; k++)
			memcpy(digests + dig_at[idx[k]], sub_dig + k * hl,
			    (size_t)hl);
	}
	if (rc == 0) {
		memset(&job, 0, sizeof(job));
		job.digests = digests;
		job.sign = sign;
		job.sigs = sigs;
		job.alg_of = alg_of;
		job.dig_at = dig_at;
		job.valid = valid;
		rc = run_ecdsa(&job, n, nthreads);
	}
out:
	free(alg_of);
	free(dig_at);
	free(idx);
	free(sub_off);
	free(sub_len);
	free(digests);
	free(sub_dig);
	return rc;
}
