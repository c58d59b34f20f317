/*
 * sha2_stream.cpp -- the streaming SHA-2 interface of src/sha2.c
 * (include/net2/sha2.h): SHA{256,384,512}{Init,Transform,Update,Pad,Final}
 * over the MI355X path.
 *
 * The context keeps src/sha2.c's layout and bookkeeping on the host
 * (state, bit count, one block of buffered bytes); every compression is a
 * BLOCKS request of the coalescer (sha2_coalesce.h), so an Update that
 * completes blocks, a Pad, or a Transform is one GPU round trip shared with
 * whatever other threads submit at the same time.  Context updates are
 * committed only after the request succeeds.
 */
#include "sha2_coalesce.h"
#include "sha2_device.h"

#include "../../include/net2/sha2.h"

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#define NET2_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

size_t block_of(int alg)
{
	return alg == 1 ? 64 : 128;
}

/* bitcount += n bits; 128-bit carry for SHA-384/512 (src/sha2.c:136-141) */
void add_bits(int alg, SHA2_CTX *c, uint64_t nbits)
{
	c->bitcount[0] += nbits;
	if (alg != 1 && c->bitcount[0] < nbits)
		c->bitcount[1]++;
}

/*
 * Bytes per coalesced request of one Update: a long Update goes through in
 * requests of at most this many bytes, so the coalescer's page-locked
 * staging stays bounded (NET2_SHA2_STREAM_CHUNK, read per call, in bytes,
 * rounded down to whole blocks; tests shrink it).
 */
size_t stream_chunk(size_t B)
{
	const char *e = getenv("NET2_SHA2_STREAM_CHUNK");
	size_t c = e != nullptr && *e != '\0' ? strtoull(e, nullptr, 10) :
	    (size_t)64 << 20;
	return std::max(c / B * B, B);
}

/*
 * state = compress(state, the whole blocks of v[0 .. nv)); all or nothing:
 * the chunks chain through a local state, committed when the last is done.
 */
int compress(int alg, void *state, const struct iovec *v, size_t nv)
{
	const size_t B = block_of(alg), S = alg == 1 ? 32 : 64;
	const size_t chunk = stream_chunk(B);
	uint8_t cur[64], next[64];
	struct iovec part[8];
	size_t i = 0, off = 0;
	memcpy(cur, state, S);
	while (i < nv) {
		/* up to `chunk` bytes of v, from v[i] + off */
		size_t np = 0, bytes = 0;
		while (i < nv && np < 8 && bytes < chunk) {
			const size_t take = std::min(v[i].iov_len - off, chunk - bytes);
			if (take != 0)
				part[np++] = { static_cast<uint8_t *>(v[i].iov_base) +
				    off, take };
			bytes += take;
			off += take;
			if (off == v[i].iov_len) {
				i++;
				off = 0;
			}
		}
		if (bytes == 0)
			continue;
		net2co::Request r = {};
		r.kind = net2co::BLOCKS;
		r.alg = alg;
		r.iov = part;
		r.iovcnt = np;
		r.state = cur;
		r.out = next;
		const int rc = net2_co_run(r);
		if (rc != 0)
			return rc;
		memcpy(cur, next, S);
	}
	memcpy(state, cur, S);
	return 0;
}

void fatal(const char *what, int rc)
{
	fprintf(stderr, "net2: %s failed on the GPU: %s (%d); the reference's "
	    "void SHA-2 calls cannot report it\n", what, strerror(rc), rc);
	abort();
}

}	/* namespace */

NET2_EXPORT int net2_sha2_ctx_init(int alg, SHA2_CTX *c)
{
	if (alg < 1 || alg > 3)
		return EINVAL;
	if (c == nullptr)
		return 0;		/* src/sha2.c:283, 569, 867 */
	if (alg == 1) {
		memcpy(c->state.st32, net2::dev::IV256, 32);
		c->bitcount[0] = 0;
	} else {
		memcpy(c->state.st64, alg == 2 ? net2::dev::IV384 :
		    net2::dev::IV512, 64);
		c->bitcount[0] = c->bitcount[1] = 0;
	}
	memset(c->buffer, 0, sizeof(c->buffer));
	return 0;
}

/* src/sha2.c:449-493 / :738-782 */
NET2_EXPORT int net2_sha2_ctx_update(int alg, SHA2_CTX *c, const void *data,
    size_t len)
{
	if (alg < 1 || alg > 3 || c == nullptr || (data == nullptr && len > 0))
		return EINVAL;
	if (len == 0)
		return 0;
	const size_t B = block_of(alg);
	const uint8_t *p = static_cast<const uint8_t *>(data);
	const size_t have = (size_t)(c->bitcount[0] >> 3) & (B - 1);
	uint8_t first[128];
	struct iovec v[2];
	size_t nv = 0, take = 0;

	if (have != 0) {
		take = std::min(B - have, len);
		if (have + take < B) {		/* still a partial block */
			memcpy(c->buffer + have, p, take);
			add_bits(alg, c, (uint64_t)take << 3);
			return 0;
		}
		memcpy(first, c->buffer, have);
		memcpy(first + have, p, take);
		v[nv++] = { first, B };
	}
	const size_t full = (len - take) / B * B;
	if (full != 0)
		v[nv++] = { const_cast<uint8_t *>(p + take), full };
	if (nv != 0) {
		const int rc = compress(alg, c->state.st32, v, nv);
		if (rc != 0)
			return rc;
	}
	/* buffer as src/sha2.c leaves it: the completed block, then the
	 * remainder over its head */
	if (have != 0)
		memcpy(c->buffer + have, p, take);
	const size_t rem = len - take - full;
	if (rem != 0)
		memcpy(c->buffer, p + take + full, rem);
	add_bits(alg, c, (uint64_t)len << 3);
	return 0;
}

/* src/sha2.c:495-543 / :784-832: one or two blocks, one request */
NET2_EXPORT int net2_sha2_ctx_pad(int alg, SHA2_CTX *c)
{
	if (alg < 1 || alg > 3 || c == nullptr)
		return EINVAL;
	const size_t B = block_of(alg), L = alg == 1 ? 8 : 16;
	uint8_t blk[2][128];
	size_t have = (size_t)(c->bitcount[0] >> 3) & (B - 1);
	int nb = 0;

	memcpy(blk[0], c->buffer, B);
	blk[0][have++] = 0x80;
	if (have > B - L) {		/* no room for the bit count */
		memset(blk[0] + have, 0, B - have);
		memcpy(blk[1], blk[0], B);
		nb = 1;
		have = 0;
	}
	uint8_t *b = blk[nb];
	memset(b + have, 0, B - L - have);
	for (int i = 0; i < 8; i++) {
		b[B - 1 - i] = (uint8_t)(c->bitcount[0] >> (8 * i));
		if (alg != 1)
			b[B - 9 - i] = (uint8_t)(c->bitcount[1] >> (8 * i));
	}
	const struct iovec v[2] = { { blk[0], B }, { blk[1], B } };
	const int rc = compress(alg, c->state.st32, v, (size_t)nb + 1);
	if (rc != 0)
		return rc;
	memcpy(c->buffer, b, B);
	return 0;
}

NET2_EXPORT int net2_sha2_ctx_final(int alg, uint8_t *digest, SHA2_CTX *c)
{
	int rc = net2_sha2_ctx_pad(alg, c);
	if (rc != 0)
		return rc;
	if (digest != nullptr) {
		/* big-endian state words (src/sha2.c:553-557, :847-850, :905-908) */
		if (alg == 1) {
			for (int i = 0; i < 8; i++)
				for (int k = 0; k < 4; k++)
					digest[4 * i + k] = (uint8_t)(c->state.st32[i] >> (24 - 8 * k));
		} else {
			for (int i = 0; i < (alg == 2 ? 6 : 8); i++)
				for (int k = 0; k < 8; k++)
					digest[8 * i + k] = (uint8_t)(c->state.st64[i] >> (56 - 8 * k));
		}
	}
	if (digest != nullptr || alg == 2)	/* SHA-384 zeroes always, :918 */
		memset(c, 0, sizeof(*c));
	return 0;
}

NET2_EXPORT int net2_sha2_ctx_transform(int alg, void *state,
    const uint8_t *block)
{
	if (alg < 1 || alg > 3 || state == nullptr || block == nullptr)
		return EINVAL;
	const struct iovec v = { const_cast<uint8_t *>(block), block_of(alg) };
	return compress(alg, state, &v, 1);
}

/* ---- the void interface of src/sha2.c ------------------------------------ */

#define NET2_SHA2_B0(PFX, ALG)                                               \
NET2_EXPORT void PFX##Init(SHA2_CTX *c)                                      \
{                                                                            \
	(void)net2_sha2_ctx_init(ALG, c);                                    \
}                                                                            \
NET2_EXPORT void PFX##Update(SHA2_CTX *c, const uint8_t *p, size_t len)      \
{                                                                            \
	int rc = net2_sha2_ctx_update(ALG, c, p, len);                       \
	if (rc != 0)                                                         \
		fatal(#PFX "Update", rc);                                    \
}                                                                            \
NET2_EXPORT void PFX##Pad(SHA2_CTX *c)                                       \
{                                                                            \
	int rc = net2_sha2_ctx_pad(ALG, c);                                  \
	if (rc != 0)                                                         \
		fatal(#PFX "Pad", rc);                                       \
}                                                                            \
NET2_EXPORT void PFX##Final(uint8_t *digest, SHA2_CTX *c)                    \
{                                                                            \
	int rc = net2_sha2_ctx_final(ALG, digest, c);                        \
	if (rc != 0)                                                         \
		fatal(#PFX "Final", rc);                                     \
}

NET2_SHA2_B0(SHA256, 1)
NET2_SHA2_B0(SHA384, 2)
NET2_SHA2_B0(SHA512, 3)

NET2_EXPORT void SHA256Transform(uint32_t state[8], const uint8_t *data)
{
	int rc = net2_sha2_ctx_transform(1, state, data);
	if (rc != 0)
		fatal("SHA256Transform", rc);
}

NET2_EXPORT void SHA384Transform(uint64_t state[8], const uint8_t *data)
{
	int rc = net2_sha2_ctx_transform(2, state, data);
	if (rc != 0)
		fatal("SHA384Transform", rc);
}

NET2_EXPORT void SHA512Transform(uint64_t state[8], const uint8_t *data)
{
	int rc = net2_sha2_ctx_transform(3, state, data);
	if (rc != 0)
		fatal("SHA512Transform", rc);
}
