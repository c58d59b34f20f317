/*
 * net2/packet.h -- the SHA-2 uses of the packet codec (types/packet.n2t)
 * on the MI355X path: IV derivation from a packet header
 * (net2_ph_to_iv, packet.n2t:100-158).  The per-datagram keyed hash of
 * net2_packet_encode/decode (packet.n2t:226-257, 410-427) is net2_hmac_dev
 * in net2/hash.h.
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
 * net2_ph_to_iv: iv = first ivlen bytes of the chain
 * iv += SHA-256(ph_network || iv) (packet.n2t:127-144), any ivlen.
 * Synchronous, one header; the SHA-256s run on the GPU.
 * 0, EINVAL, ENOMEM, ENODEV or EIO.
 */
int net2_ph_to_iv(const struct net2_packet_header *ph, size_t ivlen,
    void *iv);

/*
 * Batched form for a whole datagram batch, device-resident: header i is
 * (d_seq[i], d_flags[i]), its IV goes to d_iv + i * ivlen.  ivlen <= 64
 * (two SHA-256 rounds; AES-256-CBC, the reference's only cipher, needs 16,
 * src/enc.c:72-73).  Asynchronous on stream.
 */
int net2_ph_to_iv_dev(const uint32_t *d_seq, const uint32_t *d_flags,
    uint64_t n, uint32_t ivlen, void *d_iv, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* NET2_PACKET_H */
