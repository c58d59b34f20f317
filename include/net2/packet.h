/*
 * net2/packet.h -- the SHA-2 uses of the packet codec (types/packet.n2t)
 * on the MI355X path: IV derivation from a packet header
 * (net2_ph_to_iv, packet.n2t:100-158), and the hash steps of
 * net2_packet_encode / net2_packet_decode (packet.n2t:341-463 / :170-336)
 * for whole bursts of datagrams under one connection's keys.
 */
#ifndef NET2_PACKET_H
#define NET2_PACKET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* struct packet_header of packet.n2t:89-95; encoded as two big-endian
 * uint32 (net2_ph_overhead = 8, packet.n2t:97). */
struct net2_packet_header {
	uint32_t	seq;
	uint32_t	flags;
};

/*
 * net2_ph_to_iv_buf: the reference's net2_ph_to_iv (a decoded header in,
 * the IV into a plain buffer; the reference's own name and prototype stay
 * the reference's, packet.n2t:100-158).  iv = first ivlen bytes of the chain
 * iv += SHA-256(ph_network || iv) (packet.n2t:127-144), any ivlen.
 * Synchronous, one header; the SHA-256s run on the GPU.
 * 0, EINVAL, ENOMEM, ENODEV or EIO.
 */
int net2_ph_to_iv_buf(const struct net2_packet_header *ph, size_t ivlen,
    void *iv);

/*
 * Batched form for a whole datagram batch, device-resident: header i is
 * (d_seq[i], d_flags[i]), its IV goes to d_iv + i * ivlen.  ivlen <= 64
 * (two SHA-256 rounds; AES-256-CBC, the reference's only cipher, needs 16,
 * src/enc.c:72-73).  Asynchronous on stream.
 */
int net2_ph_to_iv_dev(const uint32_t *d_seq, const uint32_t *d_flags,
    uint64_t n, uint32_t ivlen, void *d_iv, void *stream);

/* Packet header flags used here (types/packet.n2t:27-28) and the result
 * codes of net2_packet_decode / _encode (:44-47, :53-56). */
#define NET2_PH_ENCRYPTED	0x00000001
#define NET2_PH_SIGNED		0x00000002
#define NET2_PDECODE_OK		0
#define NET2_PDECODE_RESOURCE	1
#define NET2_PDECODE_BAD	2
#define NET2_PDECODE_UNSAFE	3
#define NET2_PENCODE_OK		0
#define NET2_PENCODE_RESOURCE	1
#define NET2_PENCODE_BAD	2
#define NET2_PENCODE_UNSAFE	3

/*
 * Device scratch (bytes, 16-byte aligned) of a burst of n datagrams.  Its
 * length-binning area comes first, at the same place for every n: one
 * workspace serves bursts of any size up to its own, and
 * net2_sha2_workspace_init / net2_sha2_workspace_stats (net2/sha2_batch.h)
 * prepare and inspect it.  A keyed burst of at most 16 datagrams per SIMD
 * of the device (16,384 on an MI355X) is hashed 1 to 16 datagrams per
 * workgroup, in one launch, without touching the workspace; a larger one
 * below 65,536 datagrams (at most one wave per SIMD) is hashed in arrival
 * order, without the binning launch (net2_sha2_burst_limits below).
 */
size_t net2_packet_burst_workspace(uint64_t n);

/*
 * Size thresholds of the keyed bursts, process-wide (diagnostics, tests and
 * A/B runs): wave_max is the largest burst hashed by the one-launch
 * small-burst form (0: never), bin_min the smallest burst whose datagrams
 * are length-binned first.  A value < 0 restores that threshold's default
 * (16 datagrams per SIMD / 65,536, or NET2_BURST_WAVE_MAX /
 * NET2_BURST_BIN_MIN when set in the environment at first use).  Results do
 * not depend on either; only the time does.  Always 0.
 */
int net2_sha2_burst_limits(int64_t wave_max, int64_t bin_min);

/*
 * RX: the hash steps of net2_packet_decode for a burst of n received
 * datagrams under one connection's rx keys, device-resident and
 * asynchronous on `stream` (one stream, no host synchronisation).
 * Datagram i = d_base[d_offsets[i] .. + d_lens[i]) as it came off the wire:
 * 8-byte header (seq, flags big-endian), then the HMAC field when
 * PH_SIGNED, then the payload.  hash_alg is the negotiated keyed hash
 * (HMAC row 4..6, key of its registry length) or 0 for none; enc_alg != 0
 * when an encryption key is negotiated, ivlen its IV length (<= 64;
 * AES-256-CBC: 16, src/enc.c:72-73).  Per datagram, as packet.n2t does:
 *   - shorter than the header: NET2_PDECODE_BAD (:196-198);
 *   - PH_SIGNED / PH_ENCRYPTED missing while the key is set:
 *     NET2_PDECODE_UNSAFE (:215-221);
 *   - PH_SIGNED: the hash field is compared with HMAC(key, rest); too
 *     short or unequal: NET2_PDECODE_BAD (:226-258);
 *   - PH_ENCRYPTED and OK: the IV for the decryption step,
 *     net2_ph_to_iv (:263-279), to d_iv + i * ivlen (d_iv may be NULL).
 * d_result[i] receives the code; d_seq / d_flags (both or neither) the
 * decoded header.  The window check, the decryption itself and the key
 * commit (:200-206, :283-313) stay with the caller.
 */
int net2_packet_decode_burst(int hash_alg, const void *hash_key,
    size_t hash_keylen, int enc_alg, uint32_t ivlen, const void *d_base,
    const uint64_t *d_offsets, const uint32_t *d_lens, uint64_t n,
    uint8_t *d_result, void *d_iv, uint32_t *d_seq, uint32_t *d_flags,
    void *d_ws, size_t ws_bytes, void *stream);

/*
 * RX under a connection's full rx key state (src/conn_keys.c): during a key
 * rollover a datagram may be sealed with the alternate key.  As
 * net2_ck_rx_key (src/conn_keys.c:447-476) decides for every datagram after
 * its header is decoded (packet.n2t:210), the kernel verifies datagram i
 * with the alternate key when alt_hash_key != NULL (an alternate key is
 * installed, NET2_CK_RX_ALT) and either its flags carry PH_ALTKEY or, unless
 * alt_no_cutoff (NET2_CK_F_NO_RX_CUTOFF), seq - rx_start >=
 * alt_cutoff - rx_start (rx_start: the window's cw_rx_start); otherwise with
 * the active key.  The alternate key is new key material under the same
 * negotiated algorithms (hash_alg, enc_alg; alt_hash_keylen must equal
 * hash_keylen).  Everything else as net2_packet_decode_burst, which is this
 * call with alt_hash_key == NULL.  Committing the alternate key
 * (net2_ck_rx_key_commit, :487-510) stays with the caller.
 */
#define NET2_PH_ALTKEY		0x80000000	/* types/packet.n2t:34 */
struct net2_burst_rx_keys {
	int hash_alg;		/* 0 or an HMAC row (4..6) */
	const void *hash_key;	/* the active key */
	size_t hash_keylen;
	int enc_alg;		/* != 0: a cipher key is set */
	const void *alt_hash_key;	/* NULL: no alternate key */
	size_t alt_hash_keylen;
	int alt_no_cutoff;
	uint32_t alt_cutoff;
	uint32_t rx_start;
};
int net2_packet_decode_burst_ck(const struct net2_burst_rx_keys *keys,
    uint32_t ivlen, const void *d_base, const uint64_t *d_offsets,
    const uint32_t *d_lens, uint64_t n, uint8_t *d_result, void *d_iv,
    uint32_t *d_seq, uint32_t *d_flags, void *d_ws, size_t ws_bytes,
    void *stream);

/*
 * TX: the hash steps of net2_packet_encode for a burst.  Datagram slot i =
 * d_base[d_offsets[i] .. + d_lens[i]) holds, on entry, 8 bytes for the
 * header, then hashlen reserved bytes when d_flags[i] has PH_SIGNED (as
 * connection.c:336-339 reserves them), then the payload -- already
 * encrypted when PH_ENCRYPTED (its IV comes from net2_ph_to_iv_dev first).
 * The flags are checked against the keys both ways (NET2_PENCODE_UNSAFE,
 * :364-370); then the header (d_seq[i], d_flags[i]) is written big-endian
 * and, when PH_SIGNED, the HMAC of the payload into the reserved field
 * (:410-443).  The transmitter picks the key before it builds a datagram
 * (net2_ck_tx_key, src/conn_keys.c:544-580, sets PH_ALTKEY), so a burst
 * under the alternate tx key is a call with that key.  A slot too short for header and field gets
 * NET2_PENCODE_RESOURCE and is left untouched.  Codes to d_result.
 */
int net2_packet_encode_burst(int hash_alg, const void *hash_key,
    size_t hash_keylen, int enc_alg, const uint32_t *d_seq,
    const uint32_t *d_flags, void *d_base, const uint64_t *d_offsets,
    const uint32_t *d_lens, uint64_t n, uint8_t *d_result, void *d_ws,
    size_t ws_bytes, void *stream);

/*
 * Host-memory bursts: the same hash steps for datagrams that live in host
 * memory -- the reference's case: each received one is a net2_buffer filled
 * by net2_sockdgram_recv (src/sockdgram.c:67-108) and decoded at
 * src/connection.c:199; each sent one is built by gather()
 * (src/connection.c:336-339, :467).  Synchronous; every pointer is host
 * memory (page-locked or pageable, any mix).  The datagrams are packed into
 * pinned staging in 64 MiB chunks (two per device in flight: pack, H2D,
 * kernels, results), sharded over every usable GPU (max_devices <= 0: all;
 * no slice under 16 MiB; the list starts at the calling thread's current
 * device, as net2_sha2_batch), each slice's thread on its GPU's NUMA node.
 * The kernels store results straight into page-locked result arrays and
 * through pinned staging into pageable ones.
 *
 * RX: datagram i = base[offsets[i] .. + lens[i]); result[i] its
 * NET2_PDECODE_* code, iv + i * ivlen its IV when OK and encrypted (iv may
 * be NULL), seq[i] / flags[i] the decoded header (both or neither) --
 * exactly net2_packet_decode_burst_ck's outputs.
 *
 * TX: slot i as for net2_packet_encode_burst, in the caller's buffer: for
 * every slot whose code is NET2_PENCODE_OK the header and (PH_SIGNED) the
 * HMAC field are written into it; the payload bytes are only read.
 *
 * 0, EINVAL, ENOMEM, ENODEV or EIO (then some results may be unset).
 */
int net2_packet_decode_burst_host(const struct net2_burst_rx_keys *keys,
    uint32_t ivlen, const void *base, const uint64_t *offsets,
    const uint32_t *lens, uint64_t n, uint8_t *result, void *iv,
    uint32_t *seq, uint32_t *flags, int max_devices);
int net2_packet_encode_burst_host(int hash_alg, const void *hash_key,
    size_t hash_keylen, int enc_alg, const uint32_t *seq,
    const uint32_t *flags, void *base, const uint64_t *offsets,
    const uint32_t *lens, uint64_t n, uint8_t *result, int max_devices);

#ifdef __cplusplus
}
#endif
#endif /* NET2_PACKET_H */
