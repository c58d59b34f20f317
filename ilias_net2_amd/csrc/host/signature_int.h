/*
 * signature_int.h -- internal to libnet2_sign.so (hidden symbols).
 */
#ifndef NET2_SIGNATURE_INT_H
#define NET2_SIGNATURE_INT_H

#include "../../../include/net2/signature.h"

/* Fill s with the signature of an already computed digest
 * (types/signature.n2t:74-100); 0 or an errno, s left empty on failure. */
int sign_digest(struct net2x_signature *s, const uint8_t *digest, size_t dlen,
    const char *hash_name, struct net2x_sign_ctx *sign);

#endif /* NET2_SIGNATURE_INT_H */
