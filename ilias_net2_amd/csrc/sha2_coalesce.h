/*
 * sha2_coalesce.h -- internal: the request coalescer behind the
 * single-message entry points (net2_hashctx_hashiov, the SHA2_CTX calls of
 * net2/sha2.h, net2_ph_to_iv).  Not installed.
 *
 * The reference hashes one payload per call on whichever threadpool worker
 * runs the job (types/signature.n2t:92,147 from src/signed_carver.c:409,311;
 * include/ilias/net2/threadpool.h:33-34).  A GPU launch per call would cost
 * one serial wave per message; instead, concurrent calls on one device join
 * an open batch, and one launch hashes the whole batch, one lane per call.
 * The first caller of a batch leads it: it launches the batch when the
 * device is idle, when the batch is full, or when the batching window has
 * passed, waits for the kernel and hands every caller its result.  No
 * thread of its own, no global lock around the launch.
 */
#ifndef NET2_SHA2_COALESCE_H
#define NET2_SHA2_COALESCE_H

#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

namespace net2co {

enum Kind {
	DIGEST = 0,	/* SHA-2 digest of the message (Init/Update/Final) */
	HMAC = 1,	/* HMAC (RFC 2104) of the message under key */
	BLOCKS = 2,	/* compress whole blocks from a given state (Transform) */
};

struct Request {
	int kind;
	int alg;		/* SHA row: 1 SHA-256, 2 SHA-384, 3 SHA-512 */
	const struct iovec *iov;	/* message (BLOCKS: whole blocks) */
	size_t iovcnt;
	const uint8_t *key;	/* HMAC: key, keylen <= block size */
	size_t keylen;
	const void *state;	/* BLOCKS: uint32_t[8] / uint64_t[8] */
	uint8_t *out;		/* digest bytes, or (BLOCKS) the new state */
};

/*
 * Run r on HIP device `ordinal` through coalescer `idx` (one per device).
 * Synchronous; thread-safe.  0, EINVAL, ENOMEM or EIO (HIP error code in
 * *hip_err).  The caller's current device is unchanged on return.
 */
int submit(size_t idx, int ordinal, const Request &r, int *hip_err);

/* Requests served and launches made by coalescer idx (0, 0 before its
 * first request). */
void stats(size_t idx, uint64_t *calls, uint64_t *launches);

}	/* namespace net2co */

/*
 * submit() on the calling thread's current HIP device if it is a gfx950,
 * else on the first one (sha2_shim.cpp); ENODEV without one.  Records the
 * HIP error of an EIO for net2_sha2_last_hip_error().
 */
int net2_co_run(const net2co::Request &r);

#endif /* NET2_SHA2_COALESCE_H */
