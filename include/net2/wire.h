/*
 * net2/wire.h -- wire encodings at the boundary of the signed-payload path
 * (SURVEY.md 8f row 4), for host callers that must interoperate with the
 * reference's encoder:
 *   - struct net2_signature { string sign_alg; string hash_alg;
 *     short_net2_buffer data; } (types/signature.n2t:48-53);
 *   - struct signed_carver_header { uint16 pl_segs; uint16 sig_segs; }
 *     (types/signed_carver_header.n2t:21-43, SIGNED_CARVER_HEADERSZ = 4).
 * Integers are big-endian (include/ilias/net2/cp.h:178-205).  Strings and
 * buffers are a big-endian uint32 length, the bytes, then zero padding so
 * length field + bytes + padding is a multiple of 8
 * (cxx_src/cp.cc:20-104).  The C definition of `short_net2_buffer` is lost
 * from the tree (its net2type generator and ctypes.c are absent); the
 * surviving C++ buffer encoding above is used for it.
 */
#ifndef NET2_WIRE_H
#define NET2_WIRE_H

#include <stddef.h>
#include <stdint.h>

#include "signature.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Bytes net2x_signature_encode needs for s. */
size_t net2x_signature_encoded_len(const struct net2x_signature *s);

/* Encode s into out (capacity *outlen; length written back). 0 / EINVAL. */
int net2x_signature_encode(const struct net2x_signature *s, void *out,
    size_t *outlen);

/*
 * Decode one signature from in[0 .. inlen) into s (allocates; free with
 * net2x_signature_deinit); *consumed = bytes used.  0, EINVAL (truncated or
 * non-zero padding), ENOMEM.
 */
int net2x_signature_decode(struct net2x_signature *s, const void *in,
    size_t inlen, size_t *consumed);

struct net2_signed_carver_header {
	uint16_t	pl_segs;
	uint16_t	sig_segs;
};

/* 4 bytes: be16 pl_segs, be16 sig_segs. */
void net2_signed_carver_header_encode(
    const struct net2_signed_carver_header *h, uint8_t out[4]);
void net2_signed_carver_header_decode(struct net2_signed_carver_header *h,
    const uint8_t in[4]);

#ifdef __cplusplus
}
#endif
#endif /* NET2_WIRE_H */
