/*
 * net2/hash.h -- the C hash registry the reference's C callers link
 * against, reconstructed from its call sites (the reference tree has the
 * calls but lost the declarations and src/hash.c; SURVEY.md 8b layer B1):
 *
 *   net2_hashmax                cneg_stage1.c:1579-1591
 *   net2_hash_getname           signature.n2t:71, cneg_stage1.c:1592,
 *                               cneg_key_xchange.c:51
 *   net2_hash_findname          signature.n2t:143, cneg_stage1.c:1777
 *   net2_hash_gethashlen        conn_negotiator.c:123,200, connection.c:338,
 *                               packet.n2t:234
 *   net2_hash_getkeylen         conn_negotiator.c:122,197,
 *                               cneg_key_xchange.c:1357
 *   net2_hashctx_hashbuf        signature.n2t:92,147, packet.n2t:246,417
 *
 * Row 0 is "nil" (no hash): connection.c:336 and packet.n2t:217,364-367
 * test `alg != 0`, and the sibling enc table puts "nil" first
 * (src/enc.c:70-74).  Names are the wire strings of the C++ layer
 * (cxx_src/hash-openssl.cc:139,154,169 and :417-429); keyed rows take a key
 * of exactly hashlen bytes (hash-openssl.cc:101, :417-429).
 *
 * net2_hashctx_hashbuf took a struct net2_buffer, whose C API is also gone
 * (include/ilias/net2/buffer.h is now the C++ ilias::buffer).  Its
 * replacement takes the iovec array that net2_buffer_peek produced at every
 * call site (e.g. src/sign.c:290-295) and writes into caller memory; the
 * hashing itself runs on the GPU through net2/sha2_batch.h.
 */
#ifndef NET2_HASH_H
#define NET2_HASH_H

#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#include "sha2_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Number of registry rows (names 0 .. net2_hashmax - 1). */
extern const int net2_hashmax;

/* Wire name of row alg, or NULL if alg is out of range. */
const char *net2_hash_getname(int alg);

/* Row whose wire name is `name`, or -1 if none. */
int net2_hash_findname(const char *name);

/* Digest length in bytes of row alg (0 for nil), or -1 if out of range. */
int net2_hash_gethashlen(int alg);

/* Required key length of row alg (0 = unkeyed), or -1 if out of range. */
int net2_hash_getkeylen(int alg);

/*
 * Hash the concatenation of iov[0 .. iovcnt) with row alg and write the
 * digest (net2_hash_gethashlen(alg) bytes) to out, which holds outlen
 * bytes.  Returns 0, EINVAL (bad row, key length or outlen; an unkeyed row
 * given a key: hash-openssl.cc:199-200,227-228), ENOMEM, ENODEV or EIO.
 * A message of any length is accepted: one longer than
 * NET2_SHA2_STREAM_CHUNK (default 64 MiB) goes to the GPU in requests of at
 * most that size.  (Only with NET2_SHA2_STREAM_CHUNK set at or above the
 * message size can a single request reach the 2^32 - 64 block limit of the
 * coalescer, ~256 GiB for SHA-256, ~512 GiB for SHA-384/512: EINVAL.)
 * nil writes nothing and returns 0.  Runs on the calling thread's current
 * HIP device if it is a gfx950, else on the first gfx950; the current
 * device is unchanged on return.
 */
int net2_hashctx_hashiov(int alg, const void *key, size_t keylen,
    const struct iovec *iov, size_t iovcnt, void *out, size_t outlen);

/*
 * Counters of the request coalescer behind the single-message calls
 * (net2_hashctx_hashiov, the SHA2_CTX calls of net2/sha2.h, net2_ph_to_iv)
 * on gfx950 device `device` (an index into the devices these calls use; -1
 * = the one the calling thread's calls go to): requests served and kernel
 * launches they took since the process started.  calls / launches is the
 * mean batch size.  Either pointer may be NULL.  0, EINVAL (no such
 * device) or ENODEV.
 */
int net2_coalesce_stats(int device, uint64_t *calls, uint64_t *launches);

/*
 * Batched keyed hash (HMAC, RFC 2104) of many packets under one key -- the
 * per-datagram authenticator of net2_packet_encode/decode
 * (types/packet.n2t:246,417) for a whole receive or transmit batch.
 * alg is an HMAC row (4..6); keylen must equal its key length; key is host
 * memory.  Layouts as net2_sha2_dev_fixed (d_offsets == NULL: packet i at
 * d_base + i * stride, fixed_len bytes) or net2_sha2_dev_var (d_offsets /
 * d_lens, optional binning workspace d_ws of net2_sha2_dev_var_workspace(n)
 * bytes).  Digests (hashlen bytes each) to d_digests.  Asynchronous on
 * stream.
 */
int net2_hmac_dev(int alg, const void *key, size_t keylen,
    const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
    uint64_t stride, uint32_t fixed_len, uint64_t n, void *d_digests,
    void *d_ws, size_t ws_bytes, void *stream);

/*
 * Batched per-datagram authenticator over datagrams laid out as hash field
 * (hashlen bytes) || message, the wire order of types/packet.n2t: TX
 * prepends HMAC(key, message) (net2_packet_encode, :410-427), RX removes the
 * first hashlen bytes as the supplied hash and compares it with the HMAC of
 * the rest (net2_packet_decode, :226-257).  Datagram i is
 * d_base[d_offsets[i] .. + d_lens[i]); alg, key, keylen and the optional
 * binning workspace as net2_hmac_dev.  Datagrams must not overlap.
 * Asynchronous on stream.
 *
 * net2_hmac_sign_dev writes each datagram's hash field in place; datagrams
 * shorter than hashlen are left untouched.
 */
int net2_hmac_sign_dev(int alg, const void *key, size_t keylen,
    void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
    uint64_t n, void *d_ws, size_t ws_bytes, void *stream);

/*
 * net2_hmac_verify_dev writes one byte per datagram to d_result: 0 if the
 * hash field equals HMAC(key, message), 1 if it does not (the
 * NET2_PDECODE_BAD of packet.n2t:254-256), 2 if the datagram is shorter
 * than hashlen (NET2_PDECODE_BAD, :240-244).
 */
int net2_hmac_verify_dev(int alg, const void *key, size_t keylen,
    const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
    uint64_t n, uint8_t *d_result, void *d_ws, size_t ws_bytes,
    void *stream);

#ifdef __cplusplus
}
#endif
#endif /* NET2_HASH_H */
