/*
 * net2/sha2.h -- the streaming SHA-2 interface of src/sha2.c (layer B0 of
 * SURVEY.md 8b), restated over the MI355X path.
 *
 * src/sha2.c:38, src/sign.c:36 and types/packet.n2t:80 include
 * include/ilias/net2/bsd_compat/sha2.h, which is absent from the reference
 * tree; this header reconstructs it from every use in src/sha2.c (OpenBSD
 * layout: the context at src/sha2.c:281-289, 568-577) and keeps the names and
 * signatures, so sign.c's fingerprint loop (src/sign.c:298-307) and
 * net2_ph_to_iv (types/packet.n2t:134-142) compile against it unchanged.
 *
 * Semantics are src/sha2.c's:
 *   - Init(NULL) does nothing (src/sha2.c:283, 569, 867);
 *   - Update(ctx, p, 0) does nothing (:455, :744); whole blocks are
 *     compressed as soon as they are complete, the rest is buffered;
 *   - Pad appends 0x80, zeros and the big-endian bit count (one or two
 *     blocks, :495-543, :784-832);
 *   - Final(digest, ctx) = Pad, store the state big-endian, zero the
 *     context; Final(NULL, ctx) keeps the padded context for SHA-256 and
 *     SHA-512 (:551-562, :840-858), while SHA-384 zeroes it regardless
 *     (:918).
 * Every compression runs on the GPU (the calling thread's current gfx950
 * device, else the first): a call that completes blocks is one coalesced
 * request (sha2_coalesce.h), so concurrent callers share launches.
 *
 * The reference functions return void and cannot fail.  Here a device
 * failure inside one of them is fatal: it prints the error and aborts,
 * rather than leave a wrong digest behind.  Callers that want to handle
 * errors use the net2_sha2_ctx_* forms below, which return 0 or an errno
 * value (EINVAL, ENOMEM, ENODEV, EIO) and leave the context unchanged on
 * failure.
 */
#ifndef NET2_SHA2_H
#define NET2_SHA2_H

#include <sys/types.h>	/* BYTE_ORDER, which src/sha2.c:89-91 requires */
#include <stddef.h>
#include <stdint.h>

/*
 * src/sha2.c marks its definitions ILIAS_NET2_LOCAL (library-internal,
 * include/ilias/net2/ilias_net2_export.h:32-33), which it takes from this
 * header's include chain; spelled exactly as there, so the two definitions
 * agree whichever comes first.  With it, the reference's own src/sha2.c
 * compiles against this header unchanged (tests/test_ref_headers.py).
 */
#ifndef ILIAS_NET2_LOCAL
#if defined(__GNUC__) || defined(__clang__)
#define ILIAS_NET2_LOCAL	__attribute__ ((visibility ("hidden")))
#else
#define ILIAS_NET2_LOCAL	/* nothing */
#endif
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define SHA256_BLOCK_LENGTH		64
#define SHA256_DIGEST_LENGTH		32
#define SHA256_DIGEST_STRING_LENGTH	(SHA256_DIGEST_LENGTH * 2 + 1)
#define SHA384_BLOCK_LENGTH		128
#define SHA384_DIGEST_LENGTH		48
#define SHA384_DIGEST_STRING_LENGTH	(SHA384_DIGEST_LENGTH * 2 + 1)
#define SHA512_BLOCK_LENGTH		128
#define SHA512_DIGEST_LENGTH		64
#define SHA512_DIGEST_STRING_LENGTH	(SHA512_DIGEST_LENGTH * 2 + 1)

/* 208 bytes, the OpenBSD SHA2_CTX layout src/sha2.c uses. */
typedef struct _SHA2_CTX {
	union {
		uint32_t	st32[8];
		uint64_t	st64[8];
	} state;
	uint64_t	bitcount[2];	/* bits hashed; [1] high word (512) */
	uint8_t		buffer[SHA512_BLOCK_LENGTH];
} SHA2_CTX;

void SHA256Init(SHA2_CTX *);
void SHA256Transform(uint32_t state[8], const uint8_t data[SHA256_BLOCK_LENGTH]);
void SHA256Update(SHA2_CTX *, const uint8_t *, size_t);
void SHA256Pad(SHA2_CTX *);
void SHA256Final(uint8_t digest[SHA256_DIGEST_LENGTH], SHA2_CTX *);

void SHA384Init(SHA2_CTX *);
void SHA384Transform(uint64_t state[8], const uint8_t data[SHA384_BLOCK_LENGTH]);
void SHA384Update(SHA2_CTX *, const uint8_t *, size_t);
void SHA384Pad(SHA2_CTX *);
void SHA384Final(uint8_t digest[SHA384_DIGEST_LENGTH], SHA2_CTX *);

void SHA512Init(SHA2_CTX *);
void SHA512Transform(uint64_t state[8], const uint8_t data[SHA512_BLOCK_LENGTH]);
void SHA512Update(SHA2_CTX *, const uint8_t *, size_t);
void SHA512Pad(SHA2_CTX *);
void SHA512Final(uint8_t digest[SHA512_DIGEST_LENGTH], SHA2_CTX *);

/*
 * Error-returning forms; alg is a registry row of net2/sha2_batch.h
 * (1 SHA-256, 2 SHA-384, 3 SHA-512).  net2_sha2_ctx_final(alg, NULL, ctx)
 * is Final(NULL, ctx) above.
 */
int net2_sha2_ctx_init(int alg, SHA2_CTX *ctx);
int net2_sha2_ctx_update(int alg, SHA2_CTX *ctx, const void *data,
    size_t len);
int net2_sha2_ctx_pad(int alg, SHA2_CTX *ctx);
int net2_sha2_ctx_final(int alg, uint8_t *digest, SHA2_CTX *ctx);
int net2_sha2_ctx_transform(int alg, void *state, const uint8_t *block);

#ifdef __cplusplus
}
#endif
#endif /* NET2_SHA2_H */
