/*
 * wire.c -- encodings of net2x_signature and signed_carver_header
 * (include/net2/wire.h has the layout and its reference citations).
 */
#include "../../../include/net2/wire.h"

#include <errno.h>
#include <stdlib.h>
#include <string.h>

#define NET2_EXPORT __attribute__((visibility("default")))

/* cxx_src/cp.cc:28-37: pad so (4 + len + pad) % 8 == 0 */
static size_t
pad_of(size_t len)
{
	return 7 - (3 + len) % 8;
}

static size_t
field_len(size_t len)
{
	return 4 + len + pad_of(len);
}

static void
put_be32(uint8_t *p, uint32_t v)
{
	p[0] = (uint8_t)(v >> 24);
	p[1] = (uint8_t)(v >> 16);
	p[2] = (uint8_t)(v >> 8);
	p[3] = (uint8_t)v;
}

static uint32_t
get_be32(const uint8_t *p)
{
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) |
	    ((uint32_t)p[2] << 8) | p[3];
}

static uint8_t *
put_field(uint8_t *p, const void *data, size_t len)
{
	put_be32(p, (uint32_t)len);
	if (len)
		memcpy(p + 4, data, len);
	memset(p + 4 + len, 0, pad_of(len));
	return p + field_len(len);
}

/* Returns the field length or 0 on a malformed field. */
static size_t
get_field(const uint8_t *p, size_t avail, const uint8_t **data,
    size_t *len)
{
	size_t l, f;

	if (avail < 4)
		return 0;
	l = get_be32(p);
	f = field_len(l);
	if (f > avail || f < l)
		return 0;
	for (size_t i = 4 + l; i < f; i++)
		if (p[i] != 0)
			return 0;
	*data = p + 4;
	*len = l;
	return f;
}

NET2_EXPORT size_t
net2x_signature_encoded_len(const struct net2x_signature *s)
{
	if (s == NULL || s->sign_alg == NULL || s->hash_alg == NULL)
		return 0;
	return field_len(strlen(s->sign_alg)) + field_len(strlen(s->hash_alg)) +
	    field_len(s->datalen);
}

NET2_EXPORT int
net2x_signature_encode(const struct net2x_signature *s, void *out,
    size_t *outlen)
{
	size_t need = net2x_signature_encoded_len(s);
	uint8_t *p = out;

	if (need == 0 || outlen == NULL || out == NULL || *outlen < need ||
	    s->datalen > UINT32_MAX || (s->data == NULL && s->datalen > 0))
		return EINVAL;
	p = put_field(p, s->sign_alg, strlen(s->sign_alg));
	p = put_field(p, s->hash_alg, strlen(s->hash_alg));
	put_field(p, s->data, s->datalen);
	*outlen = need;
	return 0;
}

static char *
strndup_field(const uint8_t *d, size_t l)
{
	char *s;

	if (memchr(d, 0, l) != NULL)		/* no embedded NULs in names */
		return NULL;
	if ((s = malloc(l + 1)) == NULL)
		return NULL;
	memcpy(s, d, l);
	s[l] = 0;
	return s;
}

NET2_EXPORT int
net2x_signature_decode(struct net2x_signature *s, const void *in,
    size_t inlen, size_t *consumed)
{
	const uint8_t *p = in, *d[3];
	size_t l[3], at = 0, f;

	if (s == NULL || (in == NULL && inlen > 0))
		return EINVAL;
	for (int k = 0; k < 3; k++) {
		if ((f = get_field(p + at, inlen - at, &d[k], &l[k])) == 0)
			return EINVAL;
		at += f;
	}
	memset(s, 0, sizeof(*s));
	s->sign_alg = strndup_field(d[0], l[0]);
	s->hash_alg = strndup_field(d[1], l[1]);
	s->data = malloc(l[2] ? l[2] : 1);
	if (s->sign_alg == NULL || s->hash_alg == NULL || s->data == NULL) {
		net2x_signature_deinit(s);
		return memchr(d[0], 0, l[0]) || memchr(d[1], 0, l[1]) ? EINVAL
		    : ENOMEM;
	}
	if (l[2])
		memcpy(s->data, d[2], l[2]);
	s->datalen = l[2];
	if (consumed != NULL)
		*consumed = at;
	return 0;
}

NET2_EXPORT void
net2_signed_carver_header_encode(const struct net2_signed_carver_header *h,
    uint8_t out[4])
{
	out[0] = (uint8_t)(h->pl_segs >> 8);
	out[1] = (uint8_t)h->pl_segs;
	out[2] = (uint8_t)(h->sig_segs >> 8);
	out[3] = (uint8_t)h->sig_segs;
}

NET2_EXPORT void
net2_signed_carver_header_decode(struct net2_signed_carver_header *h,
    const uint8_t in[4])
{
	h->pl_segs = (uint16_t)((in[0] << 8) | in[1]);
	h->sig_segs = (uint16_t)((in[2] << 8) | in[3]);
}
