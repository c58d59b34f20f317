/*
 * sign.c -- ECDSA signature contexts over OpenSSL (host side of the signed
 * payload path).  Behaviour follows the reference's src/sign.c: algorithm
 * table with one "ecdsa" row (:164-169), PEM key loading (:324-420), the
 * digest signed as is with a DER ECDSA-Sig out (:478-516), validation
 * returning 1/0 (:518-563), the public key as an uncompressed point
 * (:580-639) and its SHA-256 fingerprint, cached (:258-320).  The
 * fingerprint's SHA-256 runs on the MI355X (net2_hashctx_hashiov).
 */
#define OPENSSL_SUPPRESS_DEPRECATED	/* EC_KEY point export, as sign.c */
#include "../../../include/net2/sign.h"
#include "../../../include/net2/hash.h"

#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include <openssl/bio.h>
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/evp.h>
#include <openssl/pem.h>

#define NET2_EXPORT __attribute__((visibility("default")))

struct net2x_sign_ctx {
	int		 alg;
	EVP_PKEY	*pkey;
	int		 is_private;
	pthread_mutex_t	 mu;		/* guards the two caches */
	uint8_t		*pub;		/* cached uncompressed point */
	size_t		 publen;
	int		 have_fp;
	uint8_t		 fp[32];	/* cached fingerprint */
};

static const char *const sign_names[] = { "ecdsa" };

NET2_EXPORT const int net2x_signmax =
    (int)(sizeof(sign_names) / sizeof(sign_names[0]));

/* The ECDSA row of the registry, by name (src/sign.c:653; test/sign.c:66,69
 * pass it to net2x_signctx_{priv,pub}new). */
NET2_EXPORT const int net2x_sign_ecdsa = 0;

NET2_EXPORT const char *
net2x_sign_getname(int alg)
{
	return alg >= 0 && alg < net2x_signmax ? sign_names[alg] : NULL;
}

NET2_EXPORT int
net2x_sign_findname(const char *name)
{
	if (name == NULL)
		return -1;
	for (int i = 0; i < net2x_signmax; i++)
		if (strcmp(sign_names[i], name) == 0)
			return i;
	return -1;
}

static struct net2x_sign_ctx *
ctx_from_pem(int alg, const void *key, size_t keylen, int priv)
{
	struct net2x_sign_ctx *s;
	EVP_PKEY *pk;
	BIO *bio;

	if (alg < 0 || alg >= net2x_signmax || key == NULL || keylen == 0 ||
	    keylen > INT32_MAX)
		return NULL;
	if ((bio = BIO_new_mem_buf(key, (int)keylen)) == NULL)
		return NULL;
	pk = priv ? PEM_read_bio_PrivateKey(bio, NULL, NULL, NULL)
	    : PEM_read_bio_PUBKEY(bio, NULL, NULL, NULL);
	BIO_free(bio);
	if (pk == NULL)
		return NULL;
	if (EVP_PKEY_get_base_id(pk) != EVP_PKEY_EC) {	/* ECDSA only */
		EVP_PKEY_free(pk);
		return NULL;
	}
	if ((s = calloc(1, sizeof(*s))) == NULL) {
		EVP_PKEY_free(pk);
		return NULL;
	}
	s->alg = alg;
	s->pkey = pk;
	s->is_private = priv;
	pthread_mutex_init(&s->mu, NULL);
	return s;
}

NET2_EXPORT struct net2x_sign_ctx *
net2x_signctx_pubnew(int alg, const void *key, size_t keylen)
{
	return ctx_from_pem(alg, key, keylen, 0);
}

NET2_EXPORT struct net2x_sign_ctx *
net2x_signctx_privnew(int alg, const void *key, size_t keylen)
{
	return ctx_from_pem(alg, key, keylen, 1);
}

NET2_EXPORT void
net2x_signctx_free(struct net2x_sign_ctx *s)
{
	if (s == NULL)
		return;
	EVP_PKEY_free(s->pkey);
	free(s->pub);
	pthread_mutex_destroy(&s->mu);
	free(s);
}

NET2_EXPORT struct net2x_sign_ctx *
net2x_signctx_clone(struct net2x_sign_ctx *o)
{
	struct net2x_sign_ctx *s;

	if (o == NULL || (s = calloc(1, sizeof(*s))) == NULL)
		return NULL;
	if (!EVP_PKEY_up_ref(o->pkey)) {
		free(s);
		return NULL;
	}
	s->alg = o->alg;
	s->pkey = o->pkey;
	s->is_private = o->is_private;
	pthread_mutex_init(&s->mu, NULL);
	pthread_mutex_lock(&o->mu);
	if (o->have_fp) {			/* the fingerprint cache travels */
		memcpy(s->fp, o->fp, sizeof(s->fp));
		s->have_fp = 1;
	}
	pthread_mutex_unlock(&o->mu);
	return s;
}

NET2_EXPORT size_t
net2x_signctx_maxmsglen(struct net2x_sign_ctx *s)
{
	return s == NULL ? 0 : (size_t)EVP_PKEY_get_size(s->pkey);
}

NET2_EXPORT const char *
net2x_signctx_name(struct net2x_sign_ctx *s)
{
	return s == NULL ? NULL : sign_names[s->alg];
}

NET2_EXPORT int
net2x_signctx_sign(struct net2x_sign_ctx *s, const void *in, size_t inlen,
    void *sig, size_t *siglen)
{
	EVP_PKEY_CTX *pc;
	int rc = -1;

	if (s == NULL || in == NULL || sig == NULL || siglen == NULL)
		return EINVAL;
	if (!s->is_private)
		return EINVAL;
	if (*siglen < net2x_signctx_maxmsglen(s))
		return EINVAL;
	if ((pc = EVP_PKEY_CTX_new(s->pkey, NULL)) == NULL)
		return ENOMEM;
	if (EVP_PKEY_sign_init(pc) == 1 &&
	    EVP_PKEY_sign(pc, sig, siglen, in, inlen) == 1)
		rc = 0;
	EVP_PKEY_CTX_free(pc);
	return rc;
}

NET2_EXPORT int
net2x_signctx_validate(struct net2x_sign_ctx *s, const void *sig,
    size_t siglen, const void *in, size_t inlen)
{
	EVP_PKEY_CTX *pc;
	int ok;

	if (s == NULL || in == NULL || sig == NULL)
		return 0;
	if (siglen > net2x_signctx_maxmsglen(s))	/* src/sign.c:527-529 */
		return 0;
	if ((pc = EVP_PKEY_CTX_new(s->pkey, NULL)) == NULL)
		return 0;
	ok = EVP_PKEY_verify_init(pc) == 1 &&
	    EVP_PKEY_verify(pc, sig, siglen, in, inlen) == 1;
	EVP_PKEY_CTX_free(pc);
	return ok;
}

/* Uncompressed EC point of the key, computed once. */
static int
pubkey_cached(struct net2x_sign_ctx *s)
{
	const EC_KEY *ek;
	const EC_GROUP *g;
	const EC_POINT *pt;
	size_t len;

	if (s->pub != NULL)
		return 0;
	if ((ek = EVP_PKEY_get0_EC_KEY(s->pkey)) == NULL ||
	    (g = EC_KEY_get0_group(ek)) == NULL ||
	    (pt = EC_KEY_get0_public_key(ek)) == NULL)
		return EINVAL;
	len = EC_POINT_point2oct(g, pt, POINT_CONVERSION_UNCOMPRESSED, NULL, 0,
	    NULL);
	if (len == 0)
		return EINVAL;
	if ((s->pub = malloc(len)) == NULL)
		return ENOMEM;
	if (EC_POINT_point2oct(g, pt, POINT_CONVERSION_UNCOMPRESSED, s->pub,
	    len, NULL) != len) {
		free(s->pub);
		s->pub = NULL;
		return EINVAL;
	}
	s->publen = len;
	return 0;
}

NET2_EXPORT int
net2x_signctx_pubkey(struct net2x_sign_ctx *s, void *out, size_t *outlen)
{
	int rc;

	if (s == NULL || outlen == NULL)
		return EINVAL;
	pthread_mutex_lock(&s->mu);
	rc = pubkey_cached(s);
	if (rc == 0) {
		if (out == NULL || *outlen < s->publen)
			rc = out == NULL ? 0 : EINVAL;
		else
			memcpy(out, s->pub, s->publen);
		*outlen = s->publen;
	}
	pthread_mutex_unlock(&s->mu);
	return rc;
}

NET2_EXPORT int
net2x_signctx_fingerprint(struct net2x_sign_ctx *s, uint8_t out[32])
{
	struct iovec iov;
	int rc;

	if (s == NULL || out == NULL)
		return EINVAL;
	pthread_mutex_lock(&s->mu);
	rc = 0;
	if (!s->have_fp) {
		rc = pubkey_cached(s);
		if (rc == 0) {
			iov.iov_base = s->pub;
			iov.iov_len = s->publen;
			rc = net2_hashctx_hashiov(NET2_HASH_SHA256, NULL, 0,
			    &iov, 1, s->fp, sizeof(s->fp));
		}
		if (rc == 0)
			s->have_fp = 1;
	}
	if (rc == 0)
		memcpy(out, s->fp, 32);
	pthread_mutex_unlock(&s->mu);
	return rc;
}
