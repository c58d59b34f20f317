/*
 * net2/signature.h -- hash-then-sign objects of the signed carver,
 * restated from types/signature.n2t:48-189 over plain buffers, plus the
 * batched forms that let net2_signed_carver_new / signctx_validate
 * (src/signed_carver.c:385-466, :265-338) hash a whole batch of payloads in
 * one GPU launch.
 *
 * struct net2x_signature mirrors the n2t type (signature.n2t:48-53):
 * { string sign_alg; string hash_alg; short_net2_buffer data; }.
 */
#ifndef NET2_SIGNATURE_H
#define NET2_SIGNATURE_H

#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#include "sign.h"

#ifdef __cplusplus
extern "C" {
#endif

struct net2x_signature {
	char		*sign_alg;	/* e.g. "ecdsa" */
	char		*hash_alg;	/* registry name, e.g. "SHA512" */
	uint8_t		*data;		/* DER signature of the digest */
	size_t		 datalen;
};

/*
 * signature.n2t:60-119: hash `to_sign` (iovec segments) with hash_alg on
 * the GPU, sign the digest.  0, EINVAL (NULL argument / unknown alg),
 * ENOMEM, or the errno of the hash or sign step.
 */
int net2x_signature_create(struct net2x_signature *s,
    const struct iovec *to_sign, size_t iovcnt, int hash_alg,
    struct net2x_sign_ctx *sign);

/*
 * signature.n2t:124-175: *valid = 0 first; EINVAL for NULL arguments or a
 * mismatching sign algorithm, EOPNOTSUPP for an unknown hash name, else 0
 * with *valid = 1 iff the signature matches.
 */
int net2x_signature_validate(const struct net2x_signature *s,
    const struct iovec *to_sign, size_t iovcnt, struct net2x_sign_ctx *sign,
    int *valid);

/* signature.n2t:177-189. */
void net2x_signature_deinit(struct net2x_signature *s);

/*
 * Batched create: payload i = base[offsets[i] .. + lens[i]) in host memory.
 * All n digests come from one net2_sha2_batch call; the n ECDSA signatures
 * are computed on `nthreads` host threads (<= 0: one per online CPU, at
 * most 64).  out[0 .. n) are initialised on success; on failure none are
 * left allocated.
 */
int net2x_signature_create_batch(struct net2x_signature *out,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lens,
    size_t n, int hash_alg, struct net2x_sign_ctx *sign, int nthreads);

/*
 * Batched validate of sigs[i] over payload i (same layout); valid[i] as in
 * net2x_signature_validate.  Signatures may name different hash algorithms;
 * each algorithm's payloads are hashed in one batch.
 */
int net2x_signature_validate_batch(const struct net2x_signature *sigs,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lens,
    size_t n, struct net2x_sign_ctx *sign, int *valid, int nthreads);

#ifdef __cplusplus
}
#endif
#endif /* NET2_SIGNATURE_H */
