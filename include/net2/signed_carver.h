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
 * the ECDSA signatures / verifications run on a few host threads.  The
 * collector is thread-safe: workq threads add requests while another
 * thread ticks.  Two forms share the tick:
 *   - hash requests (net2_sc_hash_req): digest out, then a caller callback
 *     -- the form the reference's signed_carver.c binds to, with ECDSA left
 *     in its own src/sign.c;
 *   - sign / validate requests over this repository's restated sign layer
 *     (net2x_, net2/sign.h; ECDSA through OpenSSL as src/sign.c:478-563).
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

/*
 * The hash-only step -- the drop-in behind the reference's own sign layer.
 *
 * In the reference, each signature's hash is taken inside
 * net2_signature_create / net2_signature_validate (types/signature.n2t:92,
 * :147, hashbuf over the payload), and the digest then goes to its own
 * net2_signctx_sign / net2_signctx_validate (include/ilias/net2/sign.h:
 * 45-50, src/sign.c:478-563).  A request here is that hash step alone:
 * payload iovecs in, digest out.  A tick hashes every request, all payloads
 * of one algorithm in one net2_sha2_batch, then calls each request's
 * `done` callback once -- on the tick's own thread or one of its helper
 * threads, so the caller's ECDSA in the callbacks runs in parallel -- with
 * rc and the digest filled in.  Nothing of the reference's sign context or
 * signature object crosses this boundary: the callback (reference code)
 * wraps the digest and calls the reference's own sign.c.  INTEGRATION.md
 * section 2 shows the binding in net2_signed_carver_new and
 * signctx_validate (src/signed_carver.c:407-432, :265-338).
 */
struct net2_sc_hash_req;
typedef void (*net2_sc_hash_cb)(struct net2_sc_hash_req *, void *arg);

struct net2_sc_hash_req {
	const struct iovec	*payload;
	size_t			 iovcnt;
	int			 hash_alg;	/* unkeyed registry row, 1..3 */
	net2_sc_hash_cb		 done;		/* NULL: no callback */
	void			*arg;		/* passed to done */
	/* out: rc 0, EINVAL (bad row or arguments, as signature.n2t:69-72),
	 * ENOMEM, or the hash path's errno; digest[0 .. digestlen) on 0 */
	int			 rc;
	uint32_t		 digestlen;
	uint8_t			 digest[64];
};

/*
 * Hash n requests at once, then run their callbacks.  Every callback runs
 * exactly once, after every digest of the tick is computed, whatever the
 * outcome (rc tells).  Returns 0 when any request succeeded, else the
 * first request's error.  nthreads as below (callbacks are spread over
 * them).  The requests are used in place: they must stay valid, and not be
 * added to another tick, until this returns.
 */
int net2_sc_hash_tick(struct net2_sc_hash_req *reqs, size_t n, int nthreads);

/* The signature step of one net2_signed_carver_new (:385-432). */
struct net2_sc_sign_req {
	const struct iovec	*payload;
	size_t			 iovcnt;
	int			 hash_alg;	/* unkeyed registry row, 1..3 */
	uint32_t		 num_signatures;
	struct net2x_sign_ctx	**signatures;	/* num_signatures contexts */
	struct net2x_signature	*out;		/* num_signatures results */
	int			 rc;		/* 0; else none of out is set */
};

/* One signctx_validate (:265-338) of a decoded signature. */
struct net2_sc_validate_req {
	const struct iovec	*payload;
	size_t			 iovcnt;
	const struct net2x_signature *sig;
	struct net2x_sign_ctx	*sctx;
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
int net2_sc_collector_add_hash(struct net2_sc_collector *,
    struct net2_sc_hash_req *);
int net2_sc_collector_add_sign(struct net2_sc_collector *,
    struct net2_sc_sign_req *);
int net2_sc_collector_add_validate(struct net2_sc_collector *,
    struct net2_sc_validate_req *);

/*
 * Run every request added since the last tick (hash, sign and validate
 * together: one GPU batch per hash algorithm); *nhash / *nsign /
 * *nvalidate (each may be NULL) receive the counts handled.  0 or an errno
 * as above.  Hash requests are handled in place (their callbacks get the
 * pointers that were added); sign / validate requests get their rc /
 * result written back.
 */
int net2_sc_collector_tick(struct net2_sc_collector *, size_t *nhash,
    size_t *nsign, size_t *nvalidate);

#ifdef __cplusplus
}
#endif
#endif /* NET2_SIGNED_CARVER_H */
