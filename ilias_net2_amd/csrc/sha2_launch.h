/*
 * sha2_launch.h -- internal interface between the C-ABI shim (sha2_shim.cpp)
 * and the kernels (sha2_kernels.hip).  Not installed; the public surface is
 * include/net2/sha2_batch.h and include/net2/hash.h.
 */
#ifndef NET2_SHA2_LAUNCH_H
#define NET2_SHA2_LAUNCH_H

#include <hip/hip_runtime.h>
#include <stdint.h>

/* Registry indices, shared with include/net2/hash.h. */
#define NET2_ALG_SHA256 1
#define NET2_ALG_SHA384 2
#define NET2_ALG_SHA512 3

/* Length bins for the variable-length path (block counts >= NBINS-1 share
 * the last bin).  65,536-byte payloads (src/carver.c:150,161) need 1,025
 * SHA-256 blocks, so every legal payload gets its own bin. */
#define NET2_SHA2_NBINS 2048

/*
 * Binning workspace (uint32 words): a 16-word header (the one-pass
 * binning's state, sha2_kernels.hip bin_onepass_kernel), the histogram in
 * two parities (2 x NBINS), the barrier words (2 x NBINS, two parities and
 * the probe stamps), then perm[n].  Header words:
 */
#define NET2_BIN_HDR 16
#define NET2_BIN_W_TAG 0	/* u64: magic << 32 | id of the launch that
				 * prepared it (0: net2_bin_ws_init) */
#define NET2_BIN_W_EPOCH 2	/* binned launches (selects the parity) */
#define NET2_BIN_W_BAD 3	/* id of a launch whose order is unusable */
#define NET2_BIN_W_ABORTS 4	/* barriers decided ABORT (timed out) */
#define NET2_BIN_W_MISMATCH 5	/* launches whose histogram total was not n */
#define NET2_BIN_W_UNPREP 6	/* launches that found the header unprepared */
#define NET2_BIN_W_TAIL 7	/* last binned launch: first position of the
				 * packets of at most 2 compressions ... */
#define NET2_BIN_W_TAILID 8	/* ... and that launch's id */
#define NET2_BIN_W_BINNED 9	/* barriers decided GO (since preparation by
				 * net2_bin_ws_init) */
/* header, the histogram's two parities, barrier words and probe stamps
 * (NET2_BIN_CTL, 4,096 words) */
#define NET2_BIN_CTL (NET2_BIN_HDR + 2 * NET2_SHA2_NBINS)
#define NET2_BIN_WS_WORDS (NET2_BIN_CTL + 2 * NET2_SHA2_NBINS)
/* Fixed-stride batch; base/out in device memory, async on s. */
hipError_t net2_launch_fixed(int alg, const uint8_t *base, uint64_t stride,
    uint32_t len, uint64_t n, uint8_t *out, hipStream_t s);

/*
 * Offset/length batch.  ws == NULL hashes in submission order (no binning);
 * otherwise ws holds NET2_BIN_WS_WORDS + n uint32 words of scratch for the
 * length-binned order.
 */
hipError_t net2_launch_var(int alg, const uint8_t *base,
    const uint64_t *offsets, const uint32_t *lens, uint64_t n, uint8_t *out,
    uint32_t *ws, hipStream_t s);

/* Prepare ws (>= NET2_BIN_WS_WORDS words) so its first binning bins, its
 * counters zeroed; an unprepared workspace hashes its first batch in
 * submission order. */
hipError_t net2_bin_ws_init(uint32_t *ws, hipStream_t s);

/*
 * Length-binned order (ws as above; perm = ws + NET2_BIN_WS_WORDS) under a
 * fresh launch id (*launch), which the hash kernel reading the order must be
 * given: it falls back to submission order when the binning found the
 * workspace inconsistent (NET2_BIN_W_BAD).
 */
hipError_t net2_bin_order(int alg, const uint32_t *lens, uint64_t n,
    uint32_t *ws, hipStream_t s, uint32_t *launch);

/*
 * Binning limits (net2_sha2_bin_limits): the persistent grid's size cap
 * (0: the device's co-resident capacity, at most 256) and the grid
 * barrier's timeout in microseconds (< 0: the default 50 ms).
 */
void net2_bin_set_limits(uint32_t grid_cap, int64_t timeout_us);

/*
 * HMAC batch (alg = 4..6).  key/keylen in host memory (keylen <= block);
 * offsets == NULL selects the fixed layout (stride, fixed_len); ws as for
 * net2_launch_var (may be NULL).  mode (variable layout only): 0 digests to
 * out; 1 sign datagrams in place (out = base: the first hashlen bytes of
 * each packet receive the HMAC of the rest); 2 verify datagrams (out[i] =
 * 0 match, 1 mismatch, 2 shorter than hashlen).
 */
#define NET2_HMAC_MODE_DIGESTS 0
#define NET2_HMAC_MODE_SIGN 1
#define NET2_HMAC_MODE_VERIFY 2
/*
 * 3: the RX burst (net2_packet_decode_burst with a hash key): offsets /
 * lens are whole wire datagrams; each lane decodes the 8-byte header, sets
 * status (NET2_PDECODE_* | 0x80 when the verdict decides), seq and flags,
 * and verifies "hash field || payload" after the header into out[i] as in
 * mode 2.  Requires burst_args.
 */
#define NET2_HMAC_MODE_BURST_RX 3
/*
 * 4: the TX burst (net2_packet_encode_burst with a hash key, out = base):
 * seq / flags are the caller's per-datagram inputs; each lane checks the
 * flags and the room, writes the 8-byte header, signs the payload into the
 * hash field after it and sets status.  Requires burst_args.
 */
#define NET2_HMAC_MODE_BURST_TX 4
struct BurstArgs {
	uint32_t *seq;		/* RX: out; TX: in */
	uint32_t *flags;	/* RX: out; TX: in */
	uint8_t *status;	/* RX: code | 0x80 (verdict pending); TX: final code */
	int enc_set;		/* a cipher key is set */
	/* RX: the connection's alternate rx key (src/conn_keys.c:447-476),
	 * same hash algorithm; used per datagram when PH_ALTKEY is set or
	 * seq - rx_start >= cutoff - rx_start (unless no_cutoff) */
	int alt;
	int alt_enc_set;
	int no_cutoff;
	uint32_t cutoff, rx_start;
	uint32_t altkey[32];	/* K' as big-endian words (the launcher turns
				 * it into midstates; unused by the kernel) */
	/* TX: when set, the datagrams in base are left as they are and the
	 * lane at binned position g writes rec + g * (hashlen + 16): the hash
	 * field (hashlen bytes, when OK), then uint32 header words as on the
	 * wire (0 unless OK), the datagram index i and its code -- status is
	 * then not written (the host burst path) */
	uint8_t *rec;
};
hipError_t net2_launch_hmac(int alg, const uint8_t *key, size_t keylen,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lens,
    uint64_t stride, uint32_t fixed_len, uint64_t n, uint8_t *out,
    uint32_t *ws, hipStream_t s, int mode = NET2_HMAC_MODE_DIGESTS,
    const BurstArgs *burst_args = nullptr);

/*
 * Small keyed bursts (net2_packet_{decode,encode}_burst with a hash key, at
 * most net2_burst_wave_max() datagrams): 1 to 16 datagrams per workgroup
 * (burst_wave_kernel) instead of 64 per wave -- the burst's time is one
 * datagram's chain either way, and the wave form shortens it by expanding
 * the message schedules in parallel.  mode NET2_HMAC_MODE_BURST_RX / _TX;
 * args as for net2_launch_hmac (RX: seq / flags receive the decoded headers,
 * either may be NULL together; TX: the inputs, and rec).  result: the final
 * code per datagram (RX; TX without rec); iv: RX IVs (ivlen <= 64; NULL or
 * 0: none); out: TX without rec, the datagrams sealed in place (== base).
 * No workspace, no separate fold / IV launch.
 */
hipError_t net2_launch_burst_wave(int alg, const uint8_t *key, size_t keylen,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lens,
    uint64_t n, const BurstArgs *args, uint8_t *result, uint8_t *iv,
    uint32_t ivlen, uint8_t *out, int mode, hipStream_t s);
/* The largest burst net2_launch_burst_wave is for on the current device:
 * 16 datagrams per SIMD, unless net2_sha2_burst_limits set a limit
 * (net2_set_burst_wave_max; < 0 clears it) or NET2_BURST_WAVE_MAX was in
 * the environment at first use (0: never). */
uint64_t net2_burst_wave_max(void);
void net2_set_burst_wave_max(int64_t v);

/*
 * Coalesced small jobs (sha2_coalesce.cpp): many independent requests from
 * host threads, each already laid out by the host as whole blocks in one
 * staging buffer.  Job j: nblk blocks at stage + data, compressed from the
 * IV of `alg` (1..3) or, with NET2_JOB_STATE, from the raw state words at
 * stage + aux; NET2_JOB_HMAC finishes with the outer hash over the
 * K' ^ opad block at stage + aux.  The final state goes to out + 64 * j as
 * raw words (uint32_t[8] or uint64_t[8], host byte order).
 */
#define NET2_JOB_STATE 0x100u
#define NET2_JOB_HMAC 0x200u
struct Net2Job {
	uint64_t data;
	uint64_t aux;
	uint32_t nblk;
	uint32_t flags;		/* alg | NET2_JOB_* */
};
/*
 * jobs [0, n256) are SHA-256, [n256, n256 + n512) SHA-384/512.  wave == 0:
 * one lane per job (throughput form, a wave per 64 jobs of a family);
 * wave != 0: one wave per job (latency form: the lanes expand the job's
 * blocks in parallel, the wave runs the rounds).
 */
/* chunk: the lane form absorbs a job in pieces of at most this many bytes
 * (a multiple of 128; its block loop counts bytes in 32 bits) */
hipError_t net2_launch_jobs(const uint8_t *stage, const Net2Job *jobs,
    uint32_t n256, uint32_t n512, uint8_t *out, uint32_t *done, int wave,
    hipStream_t s, uint32_t chunk = 0x80000000u);

/*
 * Packet bursts (net2_packet_{encode,decode}_burst): per-datagram header
 * bookkeeping (prep) and the fold of HMAC verdicts + IV derivation (final);
 * see sha2_kernels.hip.
 */
hipError_t net2_launch_burst_prep(uint8_t *base, const uint64_t *offsets,
    const uint32_t *lens, uint64_t n, int encode, int hash_set, int enc_set,
    uint32_t hashlen, const uint32_t *seq_in, const uint32_t *flags_in,
    uint32_t *seq_out, uint32_t *flags_out, uint64_t *sub_off,
    uint32_t *sub_len, uint8_t *status, hipStream_t s);
/* final: seq_out / flags_out (may be NULL) receive copies of the decoded
 * headers (the host burst path: stores into mapped host memory) */
hipError_t net2_launch_burst_final(uint64_t n, const uint8_t *status,
    const uint8_t *verdict, const uint32_t *seq, const uint32_t *flags,
    uint32_t ivlen, uint8_t *iv, uint8_t *result, hipStream_t s,
    uint32_t *seq_out = nullptr, uint32_t *flags_out = nullptr);

/* Packet-header IVs (ivlen <= 64): out = n x ivlen bytes. */
hipError_t net2_launch_ph_iv(const uint32_t *seq, const uint32_t *flags,
    uint64_t n, uint32_t ivlen, uint8_t *out, hipStream_t s);

#endif /* NET2_SHA2_LAUNCH_H */
