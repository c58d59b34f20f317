/*
 * sha2_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's SHA-2 path (nahratzah/ilias_net2
 * src/sha2.c) used as the parity checker for the HIP kernels.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product (ilias_net2_amd/libnet2_sha2.so) never links or calls it.
 *
 * Parity pin: the reference's own known-answer tests (test/hash.cc:21-48,
 * SHA-256/384/512 of "Luke, I am your father.") plus FIPS 180-4 example
 * vectors; cross-checked against Python hashlib (independent).  The
 * reference src/sha2.c itself is unbuildable in this image (it includes
 * include/ilias/net2/bsd_compat/sha2.h, which is absent from the tree), so
 * no oracle/_ref build exists -- see DESIGN.md "Oracle".
 *
 * The context layout mirrors the SHA2_CTX the reference uses
 * (src/sha2.c:281-289, 568-577): a state union of 8 x u32 / 8 x u64, a
 * two-word bit counter and a 128-byte partial-block buffer.
 */
#ifndef NET2_SHA2_ORACLE_H
#define NET2_SHA2_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_SHA256_BLOCK 64
#define ORACLE_SHA256_DIGEST 32
#define ORACLE_SHA384_BLOCK 128
#define ORACLE_SHA384_DIGEST 48
#define ORACLE_SHA512_BLOCK 128
#define ORACLE_SHA512_DIGEST 64

typedef struct oracle_sha2_ctx {
	union {
		uint32_t w32[8];
		uint64_t w64[8];
	} st;
	uint64_t bits[2];	/* [0] low 64 bits of the bit length, [1] high */
	uint8_t  blk[ORACLE_SHA512_BLOCK];
} oracle_sha2_ctx;

/* Streaming API, same call semantics as src/sha2.c's SHA{256,384,512}*. */
void oracle_sha256_init(oracle_sha2_ctx *);
void oracle_sha256_update(oracle_sha2_ctx *, const uint8_t *, size_t);
void oracle_sha256_pad(oracle_sha2_ctx *);
void oracle_sha256_final(uint8_t *digest, oracle_sha2_ctx *);
void oracle_sha256_transform(uint32_t st[8], const uint8_t blk[64]);
/* the SHA2_UNROLL_TRANSFORM form (src/sha2.c:316-370); same result */
void oracle_sha256_transform_unrolled(uint32_t st[8], const uint8_t blk[64]);

void oracle_sha512_init(oracle_sha2_ctx *);
void oracle_sha512_update(oracle_sha2_ctx *, const uint8_t *, size_t);
void oracle_sha512_pad(oracle_sha2_ctx *);
void oracle_sha512_final(uint8_t *digest, oracle_sha2_ctx *);
void oracle_sha512_transform(uint64_t st[8], const uint8_t blk[128]);
/* the SHA2_UNROLL_TRANSFORM form (src/sha2.c:605-659); same result */
void oracle_sha512_transform_unrolled(uint64_t st[8], const uint8_t blk[128]);

void oracle_sha384_init(oracle_sha2_ctx *);
void oracle_sha384_update(oracle_sha2_ctx *, const uint8_t *, size_t);
void oracle_sha384_pad(oracle_sha2_ctx *);
void oracle_sha384_final(uint8_t *digest, oracle_sha2_ctx *);

/*
 * One-shot digest.  alg: 1 = SHA-256, 2 = SHA-384, 3 = SHA-512 (the
 * registry indices of include/net2/hash.h).  Returns the digest length or
 * -1 for an unknown alg.
 */
int oracle_sha2_digest(int alg, const uint8_t *msg, size_t len, uint8_t *out);

/*
 * Batched one-shot digests over n independent packets, the CPU statement of
 * what net2_sha2_batch computes.  If offsets == NULL packet i starts at
 * base + i * stride and has length fixed_len; otherwise it starts at
 * base + offsets[i] and has length lens[i].  Digest i is written at
 * out + i * digest_len.  nthreads > 1 splits [0, n) into contiguous slices
 * run on pthreads.  Returns 0, or -1 for an unknown alg.
 */
int oracle_sha2_batch(int alg, const uint8_t *base, const uint64_t *offsets,
    const uint32_t *lens, uint64_t stride, uint32_t fixed_len, size_t n,
    uint8_t *out, int nthreads);
/* Same, with unrolled != 0 running the unrolled transforms (the reference's
 * SHA2_UNROLL_TRANSFORM build) -- the second CPU baseline of SURVEY.md 8(d). */
int oracle_sha2_batch_ex(int alg, const uint8_t *base, const uint64_t *offsets,
    const uint32_t *lens, uint64_t stride, uint32_t fixed_len, size_t n,
    uint8_t *out, int nthreads, int unrolled);

/*
 * HMAC (RFC 2104) over one message, for the keyed rows (alg 4..6 =
 * HMAC-SHA256/384/512) of the registry.  Follows what
 * cxx_src/hash-openssl.cc:285-431 delegates to OpenSSL HMAC.
 */
int oracle_hmac_digest(int alg, const uint8_t *key, size_t keylen,
    const uint8_t *msg, size_t len, uint8_t *out);

/*
 * IV derivation from a packet header (types/packet.n2t:100-158): the header
 * encoded as two big-endian uint32 (seq, flags); iv grows by SHA-256(ph ||
 * iv) until it holds ivlen bytes.
 */
int oracle_ph_to_iv(uint32_t seq, uint32_t flags, size_t ivlen, uint8_t *iv);

/*
 * Threaded batch forms (each item independent), so full-size GPU tests
 * check every result against the oracle.  HMAC over a batch under one key
 * (alg 4..6, layouts as oracle_sha2_batch); ph_to_iv of n headers into
 * iv + i * ivlen; the hash steps of net2_packet_decode / _encode
 * (types/packet.n2t:170-336 / :341-463) over a burst, as
 * net2_packet_decode_burst_ck / net2_packet_encode_burst define it
 * (alt_key NULL: no alternate rx key).  0, or -1 for a bad alg.
 */
int oracle_hmac_batch(int alg, const uint8_t *key, size_t keylen,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lens,
    uint64_t stride, uint32_t fixed_len, size_t n, uint8_t *out,
    int nthreads);
int oracle_ph_to_iv_batch(const uint32_t *seq, const uint32_t *flags,
    size_t n, size_t ivlen, uint8_t *iv, int nthreads);
int oracle_packet_decode_batch(int hash_alg, const uint8_t *key,
    size_t keylen, const uint8_t *alt_key, size_t alt_keylen,
    int alt_no_cutoff, uint32_t alt_cutoff, uint32_t rx_start, int enc_set,
    size_t ivlen, const uint8_t *base, const uint64_t *offsets,
    const uint32_t *lens, size_t n, uint8_t *result, uint8_t *iv,
    uint32_t *seq_out, uint32_t *flags_out, int nthreads);
int oracle_packet_encode_batch(int hash_alg, const uint8_t *key,
    size_t keylen, int enc_set, const uint32_t *seq, const uint32_t *flags,
    uint8_t *base, const uint64_t *offsets, const uint32_t *lens, size_t n,
    uint8_t *result, int nthreads);

#ifdef __cplusplus
}
#endif
#endif /* NET2_SHA2_ORACLE_H */
