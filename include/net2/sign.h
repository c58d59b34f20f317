/*
 * net2/sign.h -- signature contexts for the signed-payload path, restated
 * over plain buffers (the reference's net2_buffer C API is gone from its
 * tree).  Mirrors include/ilias/net2/sign.h:27-61 of the reference: same
 * argument meaning and return conventions, but under the net2x_ prefix and
 * its own context type (struct net2x_sign_ctx).  Its prototypes take plain
 * buffers where the reference's take struct net2_buffer, so it must not
 * export the reference's names: a process linking the reference's own
 * src/sign.c next to libnet2_sign.so keeps both (tests/test_ref_headers.py
 * checks that no shipped library exports a reference name with another
 * prototype).  The drop-in behind the reference's signed_carver is the
 * hash-only tick of net2/signed_carver.h, which leaves ECDSA to the
 * reference's own sign.c; this restatement is the batteries-included form
 * used by tests/c/test_sign.c and bench.py's C1 leg.
 *
 * ECDSA (the reference's only algorithm, src/sign.c:164-166) runs on the
 * host through OpenSSL exactly as src/sign.c:478-563 does (the digest is
 * signed as is, DER ECDSA-Sig out).  The one SHA-2 use of src/sign.c, the
 * public-key fingerprint (src/sign.c:258-320), is computed by the MI355X
 * path (net2_hashctx_hashiov).
 */
#ifndef NET2_SIGN_H
#define NET2_SIGN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct net2x_sign_ctx;

/* Number of signature algorithms (1: "ecdsa"), src/sign.c:164-169. */
extern const int net2x_signmax;

/* The ECDSA row (include/ilias/net2/sign.h:61, src/sign.c:653): 0. */
extern const int net2x_sign_ecdsa;

const char *net2x_sign_getname(int alg);
int net2x_sign_findname(const char *name);

/* New context from a PEM public / private key; NULL on failure
 * (src/sign.c:135-179). */
struct net2x_sign_ctx *net2x_signctx_pubnew(int alg, const void *key,
    size_t keylen);
struct net2x_sign_ctx *net2x_signctx_privnew(int alg, const void *key,
    size_t keylen);
void net2x_signctx_free(struct net2x_sign_ctx *);
struct net2x_sign_ctx *net2x_signctx_clone(struct net2x_sign_ctx *);

/* Largest signature (= ECDSA_size), src/sign.c:470-477. */
size_t net2x_signctx_maxmsglen(struct net2x_sign_ctx *);

/*
 * Sign `in` (a digest) into sig[0 .. *siglen); *siglen holds the capacity
 * on entry (>= net2x_signctx_maxmsglen).  0, EINVAL, ENOMEM or -1 on an
 * OpenSSL failure (src/sign.c:196-205, 478-516).
 */
int net2x_signctx_sign(struct net2x_sign_ctx *, const void *in, size_t inlen,
    void *sig, size_t *siglen);

/* 1 if sig is a valid signature of `in`, else 0 (src/sign.c:208-215,
 * 518-563). */
int net2x_signctx_validate(struct net2x_sign_ctx *, const void *sig,
    size_t siglen, const void *in, size_t inlen);

const char *net2x_signctx_name(struct net2x_sign_ctx *);

/*
 * Public key as an uncompressed EC point (src/sign.c:580-639).  *outlen
 * holds the capacity on entry, the length on return; 0 / EINVAL / ENOMEM.
 */
int net2x_signctx_pubkey(struct net2x_sign_ctx *, void *out, size_t *outlen);

/*
 * SHA-256 of the public key (src/sign.c:258-320), cached in the context,
 * computed on the GPU.  0, or the errno of the hash path.
 */
int net2x_signctx_fingerprint(struct net2x_sign_ctx *, uint8_t out[32]);

#ifdef __cplusplus
}
#endif
#endif /* NET2_SIGN_H */
