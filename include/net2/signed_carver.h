/*
 * net2/signed_carver.h -- the hashing and signing steps of the signed
 * carver (src/signed_carver.c), batched per workq tick.
 *
 * The reference creates, for every new signed carver, one signature per
 * sign context over the whole payload (net2_signed_carver_new,
 * src/signed_carver.c:407-432: net2_signature_create per context, so the
 * payload is hashed once per context), and validates each received
 * (payload, signature) pair in a promise-combine callback on a threadpool
 * worker (signed_combiner_check / signctx_validate, :344-367 / :265-338).
 *
 * Here the carvers and combiner checks that come up in one tick are
 * collected and handled together: every payload is hashed once, all
 * payloads of one hash algorithm in one GPU batch (net2_sha2_batch), and
 * the ECDSA signatures / verifications (OpenSSL, as src/sign.c:478-563)
 * run on a few host threads.  The collector is thread-safe: workq threads
 * add requests while another thread ticks.
 *
 * Payloads are iovec arrays (what net2_buffer_peek yields, src/sign.c:
 * 290-295) and must stay valid until the tick that handles them returns.
 */
#ifndef NET2_SIGNED_CARVER_H
#define NET2_SIGNED_CARVER_H

#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#include "sign.h"
#include "signature.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The signature step of one net2_signed_carver_new (:385-432). */
struct net2_sc_sign_req {
	const struct iovec	*payload;
	size_t			 iovcnt;
	int			 hash_alg;	/* unkeyed registry row, 1..3 */
	uint32_t		 num_signatures;
	struct net2_sign_ctx	**signatures;	/* num_signatures contexts */
	struct net2_signature	*out;		/* num_signatures results */
	int			 rc;		/* 0; else none of out is set */
};

/* One signctx_validate (:265-338) of a decoded signature. */
struct net2_sc_validate_req {
	const struct iovec	*payload;
	size_t			 iovcnt;
	const struct net2_signature *sig;
	struct net2_sign_ctx	*sctx;
	/* the promise outcome: 0 (finok, :316-317), EINVAL (signature does
	 * not match, :318-319) or EIO (could not be validated: unknown hash,
	 * wrong sign algorithm, resource failure, :333-336) */
	int			 result;
};

/*
 * Handle n carvers' signature steps at once.  Per request rc: 0, EINVAL
 * (bad hash row or arguments), ENOMEM, or the error of the GPU hash / the
 * sign step.  Returns 0 when any request succeeded -- the per-request
 * values are then the outcome, e.g. a SHA-512 group can fail while the
 * SHA-256 group of the same tick signs -- or, when every request failed,
 * the first request's error (each rc carries its own).  nthreads <= 0: one per online CPU, at most 64.
 */
int net2_signed_carver_sign_tick(struct net2_sc_sign_req *reqs, size_t n,
    int nthreads);

/* Handle n combiner checks at once; result per request as above (a check
 * that ran and found the signature invalid, EINVAL, counts as handled). */
int net2_signed_combiner_validate_tick(struct net2_sc_validate_req *reqs,
    size_t n, int nthreads);

/* The collector: add from any thread, tick from one. */
struct net2_sc_collector;

struct net2_sc_collector *net2_sc_collector_new(int nthreads);
void net2_sc_collector_free(struct net2_sc_collector *);
int net2_sc_collector_add_sign(struct net2_sc_collector *,
    struct net2_sc_sign_req *);
int net2_sc_collector_add_validate(struct net2_sc_collector *,
    struct net2_sc_validate_req *);

/*
 * Run every request added since the last tick (sign and validate
 * together: one GPU batch per hash algorithm); *nsign / *nvalidate (may be
 * NULL) receive the counts handled.  0 or an errno as above.
 */
int net2_sc_collector_tick(struct net2_sc_collector *, size_t *nsign,
    size_t *nvalidate);

#ifdef __cplusplus
}
#endif
#endif /* NET2_SIGNED_CARVER_H */
