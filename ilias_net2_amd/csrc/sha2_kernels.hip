/*
 * sha2_kernels.hip -- batched SHA-256/384/512 digests for gfx950 (MI355X).
 *
 * The reference hashes one payload at a time on a host thread:
 * SHA{256,512}Init -> Update (per iovec) -> Final (src/sha2.c:280-563,
 * :566-919), called from net2_signature_create/validate
 * (types/signature.n2t:92,147) and net2_signctx_fingerprint
 * (src/sign.c:298-307).  Here one wavefront lane owns one packet and runs
 * Init/Update/Pad/Final for it entirely in registers; a launch covers a whole
 * batch of independent packets.
 *
 * Layouts (device memory):
 *   fixed  : packet i = base[i * stride .. i * stride + len)
 *   var    : packet i = base[offsets[i] .. offsets[i] + lens[i])
 *   digests: digest i at out + i * digest_len (32 / 48 / 64 bytes)
 * Variable-length batches are length-binned first (bin_* kernels below) so
 * that the lanes of a wave share a block count: an unbinned {64,512,1500} B
 * mix runs every wave at the 24-block worst case, binned at the average.
 *
 * The block loop is VALU-bound (~1,400 integer ops per 64-byte SHA-256
 * block), so the memory side only has to keep loads in flight: each lane
 * prefetches block k+1 while compressing block k.
 */
#include "sha2_device.h"
#include "sha2_launch.h"

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>

namespace net2 {
namespace dev {

/* ---- hash traits ------------------------------------------------------ */

/*
 * Per-kernel code-shape choices (each measured):
 *   ASM: round bodies as ordered asm blocks (round256_asm, sha2_device.h);
 *   U2:  the two-block ping-pong block loop (absorb below);
 *   PAIR: the pair loop -- both 64-byte blocks of a 128-byte line requested
 *         together, one pair ahead (absorb below);
 *   DRAIN: issue priority while the grid drains (prio_remaining);
 *   GLDS: LDS-DMA staging of the next block (absorb);
 *   PREFETCH: block k+1 in flight while block k is compressed.
 * Alternatives that lost their A/B (the evidence stays
 * under profiles/) are removed from the source, not kept behind switches.
 */
template <bool ASM_, bool U2_, bool PAIR_ = false, bool DRAIN_ = false>
struct Sha256T {
	static constexpr bool ASM = ASM_;
	static constexpr bool U2 = U2_;
	static constexpr bool PAIR = PAIR_;
	static constexpr bool DRAIN = DRAIN_;	/* prio_remaining */
	static constexpr bool GLDS = false;	/* absorb: LDS-DMA staging */
	typedef uint32_t word;
	static constexpr int BLOCK = 64;	/* bytes per block */
	static constexpr int NW32 = 16;		/* 32-bit words per block */
	static constexpr int LENBYTES = 8;	/* trailing length field */
	static constexpr int DLEN = 32;
	/* prefetch block k+1 during block k: 16 VGPRs, still 8 waves/SIMD */
	static constexpr bool PREFETCH = true;
	typedef uint32_t State[8];

	__device__ __forceinline__ static void init(State &st, int)
	{
#pragma unroll
		for (int i = 0; i < 8; i++)
			st[i] = IV256[i];
	}
	__device__ __forceinline__ static void compress(State &st,
	    uint32_t (&b)[16])
	{
		compress256<ASM>(st, b);
	}
	/* Store state big-endian (src/sha2.c:553-557) as 32-bit words. */
	__device__ __forceinline__ static void out_words(const State &st,
	    uint32_t (&o)[16], int)
	{
#pragma unroll
		for (int i = 0; i < 8; i++)
			o[i] = bswap32(st[i]);
	}
};
/*
 * Every SHA-256 kernel takes the asm rounds, the two-block loop and the
 * pair loop (fixed kernel: 92 VGPRs; variable-length kernel: 96, C3 +0.7 %
 * with the pair loop, profiles/round1/var_pair_ab.txt; C3 452 against
 * 463 us with the asm rounds, profiles/round2/var_asm_ab.txt); the HMAC
 * kernels in every mode (launch_hmac_var_mode).
 */
typedef Sha256T<true, true, true> Sha256;	/* fixed, variable, HMAC */
typedef Sha256 Sha256V;
typedef Sha256 Sha256H;

struct Sha512 {
	static constexpr bool ASM = false;
	/* no prefetch: a 128-byte block would cost 32 VGPRs and a wave per
	 * SIMD (the two-block ping-pong: -1.4 %, with 5 waves -18 %,
	 * profiles/round2/fixed512_prefetch_ab.txt) */
	static constexpr bool U2 = false;
	static constexpr bool PAIR = false;	/* a 128-byte block is a whole line */
	/* drain priority (prio_remaining): the fixed kernel only, C4 +1.2 %
	 * (profiles/round2/drain_prio_ab.txt) */
	static constexpr bool DRAIN = true;
	static constexpr bool GLDS = false;
	typedef uint64_t word;
	static constexpr int BLOCK = 128;
	static constexpr int NW32 = 32;
	static constexpr int LENBYTES = 16;
	static constexpr int DLEN = 64;		/* 48 for SHA-384 */
	static constexpr bool PREFETCH = false;
	typedef uint64_t State[8];

	__device__ __forceinline__ static void init(State &st, int is384)
	{
#pragma unroll
		for (int i = 0; i < 8; i++)
			st[i] = is384 ? IV384[i] : IV512[i];
	}
	__device__ __forceinline__ static void compress(State &st,
	    uint32_t (&b)[32])
	{
		uint64_t w[16];
#pragma unroll
		for (int i = 0; i < 16; i++)
			w[i] = mk64(b[2 * i + 1], b[2 * i]);
		compress512(st, w);
	}
	__device__ __forceinline__ static void out_words(const State &st,
	    uint32_t (&o)[16], int)
	{
#pragma unroll
		for (int i = 0; i < 8; i++) {
			o[2 * i] = bswap32(hi32(st[i]));
			o[2 * i + 1] = bswap32(lo32(st[i]));
		}
	}
};

/*
 * SHA-512 for the variable-length kernel: no prefetch -- neither the
 * two-block ping-pong (136-140 VGPRs, 3 waves; +1.9 % on c3_512 on one box,
 * -1.3 % on another, -3 to -4 % on the HMAC-SHA512 MTU configs and both
 * bursts) nor LDS-DMA staging (-1.4 to -2.8 %, profiles/round3/glds_*_ab.txt).
 */
struct Sha512V : Sha512 {
	static constexpr bool DRAIN = false;
};
/* ... for the lane-per-job kernel of the coalescer, whose blocks come over
 * PCIe from zero-copy staging: the next block's load is in flight while one
 * is compressed (64 threads of 1 KiB SHA-512 calls: 431 k against 399 k
 * calls/s, profiles/round2/coalesce_job512_prefetch_ab.txt) ... */
struct Sha512J : Sha512 {
	static constexpr bool DRAIN = false;
	static constexpr bool U2 = true;
	static constexpr bool PREFETCH = true;
};
/* ... for the variable-length HMAC kernels (as Sha512V) ... */
struct Sha512H : Sha512 {
	static constexpr bool DRAIN = false;
};
/* ... and for the fixed-layout HMAC-SHA512 kernel: drain priority kept, the
 * next block fetched with LDS-DMA (global_load_lds) into a per-wave LDS slab
 * while the current one is compressed -- a prefetch that costs no VGPRs
 * (absorb below).  96 VGPRs, its ~35 KB of slabs per workgroup hold it at
 * 4 waves per SIMD; without them it runs 5 waves at 95 VGPRs and measured
 * 0.7 % slower (profiles/round5/ab_hostmid_box2.txt) */
struct Sha512HF : Sha512 {
	static constexpr bool GLDS = true;
};

/* ---- message loading ------------------------------------------------- */

/*
 * Address modes.  A16: every packet start in the wave is 16-byte aligned, a
 * block is NW32/4 global_load_dwordx4.  A4: dword-aligned starts (packed
 * packets whose lengths are multiples of 4, e.g. 1,500-byte datagrams), a
 * block is NW32 global_load_dword.  A1: arbitrary byte alignment; the
 * block is read as NW32 + 1 naturally aligned dwords (the extra one only
 * when misaligned, so no dword outside the packet's own bytes is touched)
 * and re-aligned with v_alignbyte_b32.
 */
enum { AMODE_A16 = 0, AMODE_A1 = 1, AMODE_A4 = 2 };
/*
 * One address path for the SHA-512 variable-length and HMAC kernels: they
 * take the A16 block loads (global_load_dwordx4 at the block start) whatever
 * the packet's alignment, relying on the unaligned access mode ROCm sets for
 * gfx9+ global memory (tools/unaligned_probe.hip: every byte offset reads
 * the right bytes on gfx950, profiles/round4/unaligned_probe.json) -- one
 * code path per kernel instead of three chosen per wave.  The tail block
 * keeps its aligned-dword reads (it never touches a byte past the packet).
 * From order-flipped A/Bs on separate boxes (profiles/round4/ab_*.txt): the
 * SHA-512 kernels gain (HMAC-SHA512 verify +2.8 %, burst RX +2 %, c3_512
 * +0.5 to +1.2 %), the SHA-256 kernels keep the three paths (HMAC-SHA256
 * verify 1.5 % and C3 0.45 % faster with them).
 */
template <class H>
struct OnePath {
	static constexpr bool value = sizeof(typename H::word) == 8;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
/*
 * Dword loads from an address rebuilt from an integer (the aligned-down
 * start of a byte-aligned packet) go through a global pointer: a plain
 * pointer would be a flat load, which may alias LDS, and in a kernel with
 * LDS-DMA in flight every flat load waits for all outstanding loads first.
 */
typedef __attribute__((address_space(1))) const uint32_t gconst_u32;

template <int NW32>
struct Raw {
	uint32_t d[NW32 + 1];
};

template <int NW32, int AMODE>
__device__ __forceinline__ void issue_block(const uint8_t *p, Raw<NW32> &r)
{
	if (AMODE == AMODE_A16) {
		const u32x4 *q = reinterpret_cast<const u32x4 *>(p);
#pragma unroll
		for (int i = 0; i < NW32 / 4; i++) {
			u32x4 v = q[i];
			r.d[4 * i] = v.x;
			r.d[4 * i + 1] = v.y;
			r.d[4 * i + 2] = v.z;
			r.d[4 * i + 3] = v.w;
		}
	} else if (AMODE == AMODE_A4) {
		const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
#pragma unroll
		for (int i = 0; i < NW32; i++)
			r.d[i] = q[i];
	} else {
		uintptr_t a = reinterpret_cast<uintptr_t>(p);
		const gconst_u32 *q = (const gconst_u32 *)(a & ~(uintptr_t)3);
#pragma unroll
		for (int i = 0; i < NW32; i++)
			r.d[i] = q[i];
		r.d[NW32] = (a & 3) ? q[NW32] : 0u;
	}
}

/* Raw little-endian dwords -> big-endian message words. */
template <int NW32, int AMODE>
__device__ __forceinline__ void finish_block(const uint8_t *p,
    const Raw<NW32> &r, uint32_t (&w)[NW32])
{
	if (AMODE == AMODE_A16 || AMODE == AMODE_A4) {
#pragma unroll
		for (int i = 0; i < NW32; i++)
			w[i] = bswap32(r.d[i]);
	} else {
		uint32_t sh = (uint32_t)reinterpret_cast<uintptr_t>(p) & 3;
#pragma unroll
		for (int i = 0; i < NW32; i++)
			w[i] = bswap32(__builtin_amdgcn_alignbyte(r.d[i + 1],
			    r.d[i], sh));
	}
}

/*
 * LDS-DMA staging (H::GLDS).  A global_load_lds instruction writes the
 * wave's 64 lane chunks to LDS lane-linearly (wave-uniform base + lane x
 * size), with no VGPR destination.  Chunk j (16 bytes) of every lane's
 * block goes to its own 1 KiB row of the wave's slab, so lane l reads its
 * block back from its own column with ds_read_b128 (consecutive lanes,
 * consecutive banks).  All address modes fetch 16-byte chunks: A16 and A4
 * from the block start (a global dwordx4 needs only dword alignment), A1
 * from the naturally aligned dword below it, plus the one dword past the
 * 32nd into a 256-byte row of its own when the start is misaligned -- the
 * bytes issue_block reads, never one outside the packet.  (Dword-wide
 * fetches, 32 per block, measured 35-42 % slower on the variable-length
 * SHA-512 kernels: every instruction touches the wave's 64 lines.)
 * One 8,448-byte slab per wave of a 256-thread workgroup.
 */
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;
#define NET2_GLDS_WORDS (33 * 64)
__shared__ uint32_t glds_slab[4 * NET2_GLDS_WORDS];

__device__ __forceinline__ uint32_t *glds_wave_slab()
{
	const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	return glds_slab + wv * NET2_GLDS_WORDS;
}

template <int NW32, int AMODE>
__device__ __forceinline__ void glds_issue(const uint8_t *p, uint32_t *slab)
{
	const uintptr_t a = reinterpret_cast<uintptr_t>(p);
	const uint8_t *q = AMODE != AMODE_A1 ? p :
	    reinterpret_cast<const uint8_t *>(a & ~(uintptr_t)3);
#pragma unroll
	for (int j = 0; j < NW32 / 4; j++)
		__builtin_amdgcn_global_load_lds((glb_void *)(q + 16 * j),
		    (lds_void *)(slab + 256 * j), 16, 0, 0);
	if (AMODE == AMODE_A1 && (a & 3))
		__builtin_amdgcn_global_load_lds((glb_void *)(q + 4 * NW32),
		    (lds_void *)(slab + 64 * NW32), 4, 0, 0);
}

/* The lane's staged block back from the slab, as issue_block leaves it. */
template <int NW32, int AMODE>
__device__ __forceinline__ void glds_read(const uint32_t *slab, Raw<NW32> &r)
{
	const uint32_t lane = threadIdx.x & 63;
	const u32x4 *s = reinterpret_cast<const u32x4 *>(slab) + lane;
#pragma unroll
	for (int j = 0; j < NW32 / 4; j++) {
		const u32x4 v = s[64 * j];
		r.d[4 * j] = v.x;
		r.d[4 * j + 1] = v.y;
		r.d[4 * j + 2] = v.z;
		r.d[4 * j + 3] = v.w;
	}
	/* the A1 dword past the 32nd; unused when the start is aligned
	 * (alignbyte by 0) */
	r.d[NW32] = AMODE == AMODE_A1 ? slab[64 * NW32 + lane] : 0u;
}

/*
 * The last data bytes q[0 .. rem) (rem < BLOCK) followed by the 0x80
 * terminator and zero fill, as big-endian words (the buffer SHA256Pad /
 * SHA512Pad build, src/sha2.c:495-526 / :784-812).  Only dwords that hold
 * packet bytes are read.
 */
template <int NW32>
__device__ __forceinline__ void tail_block(const uint8_t *q, uint32_t rem,
    uint32_t (&w)[NW32])
{
	uintptr_t a = reinterpret_cast<uintptr_t>(q);
	uint32_t sh = (uint32_t)a & 3;
	const gconst_u32 *al = (const gconst_u32 *)(a - sh);
	uint32_t d[NW32 + 1];
#pragma unroll
	for (int j = 0; j <= NW32; j++)
		d[j] = (uint32_t)(4 * j) < sh + rem ? al[j] : 0u;
#pragma unroll
	for (int i = 0; i < NW32; i++) {
		uint32_t x = bswap32(__builtin_amdgcn_alignbyte(d[i + 1], d[i],
		    sh));
		int kk = (int)rem - 4 * i;	/* message bytes in this word */
		if (kk < 4) {
			uint32_t keep = kk > 0 ? ~(0xffffffffu >> (8 * kk)) : 0u;
			uint32_t mark = kk >= 0 ? 0x80000000u >> (8 * kk) : 0u;
			x = (x & keep) | mark;
		}
		w[i] = x;
	}
}

/* Digest store: 16-byte vector stores when aligned, bytes otherwise. */
template <int DLEN>
__device__ __forceinline__ void store_digest(uint8_t *o, const uint32_t (&v)[16])
{
	if ((reinterpret_cast<uintptr_t>(o) & 15) == 0) {
		uint4 *q = reinterpret_cast<uint4 *>(o);
#pragma unroll
		for (int i = 0; i < DLEN / 16; i++)
			q[i] = make_uint4(v[4 * i], v[4 * i + 1], v[4 * i + 2],
			    v[4 * i + 3]);
	} else {
#pragma unroll
		for (int i = 0; i < DLEN / 4; i++) {
			uint32_t x = v[i];
			o[4 * i] = (uint8_t)x;
			o[4 * i + 1] = (uint8_t)(x >> 8);
			o[4 * i + 2] = (uint8_t)(x >> 16);
			o[4 * i + 3] = (uint8_t)(x >> 24);
		}
	}
}

/*
 * Pin a finished state before a lane-conditional use (`if (live) store`):
 * otherwise the compiler sinks the last compression into the branch and
 * leaves its LDS constant reads (SHA-512) above it, all live at once.
 */
template <class H>
__device__ __forceinline__ void materialize(const typename H::State &st)
{
#pragma unroll
	for (int i = 0; i < 8; i++)
		asm volatile("" ::"v"(st[i]));
}

/*
 * Issue priority while a grid drains (H::DRAIN: the fixed SHA-512 kernel;
 * not on the byte-aligned load path).
 * The SIMD's VALU arbiter serves the oldest wave first, so when the grid's
 * last generation of waves is dispatched, the youngest waves -- those with
 * the most blocks left -- progress last and finish alone, at one wave's
 * issue rate.  In the workgroups of the grid's last kPrioGen x 256 (two
 * per CU), a wave's priority follows the work it has left (s_setprio 3..0
 * as its remaining blocks fall below 12 / 6 / 2), so the waves of a SIMD
 * end closer together.  C4 +1.0 % (six alternations on two boxes; one or
 * three / four generations: +0.7 % / flat), C2 flat
 * (profiles/round2/drain_prio_ab.txt).  The same priority in every wave of
 * the grid measured slower (C2 -5 %, C4 -6 %, C3 -1 %,
 * profiles/round2/prio_ab.txt): the age order keeps the waves of a SIMD out
 * of phase, so their loads do not all wait at once.
 */
constexpr unsigned kPrioGen = 2;
template <bool DRAIN>
__device__ __forceinline__ void prio_remaining(uint32_t rem_blocks)
{
	if (!DRAIN)
		return;
	if (gridDim.x < 4 * 256 * kPrioGen ||
	    blockIdx.x + 256 * kPrioGen < gridDim.x)
		return;
	const uint32_t r = __builtin_amdgcn_readfirstlane(rem_blocks);
	if (r >= 12)
		__builtin_amdgcn_s_setprio(3);
	else if (r >= 6)
		__builtin_amdgcn_s_setprio(2);
	else if (r >= 2)
		__builtin_amdgcn_s_setprio(1);
	else
		__builtin_amdgcn_s_setprio(0);
}

/*
 * Whole-message digest for one lane.  nfull full blocks stream from p with
 * a one-block prefetch; then the generic tail (data remainder + 0x80 +
 * length, one or two blocks), or -- when the caller knows every message of
 * the launch is a multiple of the block size -- the constant padding block
 * whose K[t] + W[t] schedule the host precomputed (kw).
 */
/*
 * SHA*Update over the len / BLOCK full blocks at p (src/sha2.c:477-485:
 * whole blocks are transformed straight from caller memory).  With
 * PREFETCH, block k+1 is loaded while block k is compressed.
 */
template <class H, int AMODE, bool PREFETCH = H::PREFETCH>
__device__ __forceinline__ void absorb(const uint8_t *p, uint32_t len,
    typename H::State &st)
{
	constexpr int NW32 = H::NW32;
	const uint32_t nfull = len / H::BLOCK;

	if constexpr (H::GLDS) {
		/*
		 * Block k+1 is requested into the wave's LDS slab (no VGPRs)
		 * once block k has been read out of it, so its memory latency
		 * runs under block k's compression.  The waits are explicit:
		 * the slab is complete after vmcnt(0), and free again once the
		 * lane's reads have returned (lgkmcnt(0)).
		 */
		uint32_t *slab = glds_wave_slab();
		if (nfull > 0)
			glds_issue<NW32, AMODE>(p, slab);
		for (uint32_t k = 0; k < nfull; k++) {
			prio_remaining<H::DRAIN && AMODE != AMODE_A1>(nfull - k);
			const uint8_t *bp = p + (size_t)k * H::BLOCK;
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			Raw<NW32> r;
			glds_read<NW32, AMODE>(slab, r);
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			if (k + 1 < nfull)
				glds_issue<NW32, AMODE>(bp + H::BLOCK, slab);
			uint32_t w[NW32];
			finish_block<NW32, AMODE>(bp, r, w);
			H::compress(st, w);
		}
	} else if (PREFETCH && H::PAIR) {
		/*
		 * Pairs of blocks (one 128-byte line of an aligned packet)
		 * requested together, one pair ahead: two pair buffers swap
		 * roles every pair, so a trip covers four blocks.  With the
		 * one-block-ahead prefetch below, a line's second half was
		 * requested one compression (~20 us) after its first, long
		 * enough for ~10 % of the lines to leave the XCD's 4 MB L2 and
		 * be fetched again; here C2 reads exactly the payload, at the
		 * same speed (92 VGPRs, 5 waves/SIMD;
		 * profiles/round1/pairload_fetch.json).
		 */
		const uint32_t npairs = nfull / 2;
		Raw<NW32> a0, a1, b0, b1;
		if (npairs > 0) {
			issue_block<NW32, AMODE>(p, a0);
			issue_block<NW32, AMODE>(p + H::BLOCK, a1);
		}
		uint32_t q = 0;
		for (; q + 2 <= npairs; q += 2) {
			prio_remaining<H::DRAIN && AMODE != AMODE_A1>(nfull - 2 * q);
			const uint8_t *bp = p + (size_t)q * 2 * H::BLOCK;
			/* (requested one compression later instead, so the first
			 * wave generation asks for one line per lane before it
			 * starts: C2 -0.3 %, HMAC-SHA256 -0.9 %,
			 * profiles/round2/pair_late_ab.txt) */
			issue_block<NW32, AMODE>(bp + 2 * H::BLOCK, b0);
			issue_block<NW32, AMODE>(bp + 3 * H::BLOCK, b1);
			uint32_t w[NW32];
			finish_block<NW32, AMODE>(bp, a0, w);
			H::compress(st, w);
			finish_block<NW32, AMODE>(bp + H::BLOCK, a1, w);
			H::compress(st, w);
			/* past the last pair: re-read pair q + 1 (in bounds, L2-hot,
			 * unused) so a0/a1 are always defined here */
			const uint8_t *np = bp + (q + 2 < npairs ? 4 : 2) * H::BLOCK;
			issue_block<NW32, AMODE>(np, a0);
			issue_block<NW32, AMODE>(np + H::BLOCK, a1);
			finish_block<NW32, AMODE>(bp + 2 * H::BLOCK, b0, w);
			H::compress(st, w);
			finish_block<NW32, AMODE>(bp + 3 * H::BLOCK, b1, w);
			H::compress(st, w);
		}
		if (q < npairs) {
			const uint8_t *bp = p + (size_t)q * 2 * H::BLOCK;
			uint32_t w[NW32];
			finish_block<NW32, AMODE>(bp, a0, w);
			H::compress(st, w);
			finish_block<NW32, AMODE>(bp + H::BLOCK, a1, w);
			H::compress(st, w);
		}
		if (nfull & 1) {
			const uint8_t *bp = p + (size_t)(nfull - 1) * H::BLOCK;
			Raw<NW32> r;
			issue_block<NW32, AMODE>(bp, r);
			uint32_t w[NW32];
			finish_block<NW32, AMODE>(bp, r, w);
			H::compress(st, w);
		}
	} else if (PREFETCH && H::U2) {
		/*
		 * Two blocks per trip with the buffers swapping roles, so the
		 * prefetched block is consumed where it landed (a one-block loop
		 * copies it over: 16 v_mov per block).
		 */
		Raw<NW32> ra, rb;
		if (nfull > 0)
			issue_block<NW32, AMODE>(p, ra);
		uint32_t k = 0;
		for (; k + 2 <= nfull; k += 2) {
			prio_remaining<H::DRAIN && AMODE != AMODE_A1>(nfull - k);
			const uint8_t *bp = p + (size_t)k * H::BLOCK;
			issue_block<NW32, AMODE>(bp + H::BLOCK, rb);
			uint32_t w[NW32];
			finish_block<NW32, AMODE>(bp, ra, w);
			H::compress(st, w);
			/*
			 * Unconditional, so ra is always (re)defined here: a
			 * conditional load makes ra a phi and brings the copies
			 * back.  Past the last block it re-reads block k + 1
			 * (in bounds, L2-hot) and the result is unused.
			 */
			issue_block<NW32, AMODE>(bp + (k + 2 < nfull ? 2 : 1) *
			    H::BLOCK, ra);
			uint32_t w2[NW32];
			finish_block<NW32, AMODE>(bp + H::BLOCK, rb, w2);
			H::compress(st, w2);
		}
		if (k < nfull) {
			uint32_t w[NW32];
			finish_block<NW32, AMODE>(p + (size_t)k * H::BLOCK, ra, w);
			H::compress(st, w);
		}
	} else if (PREFETCH) {
		Raw<NW32> cur;
		if (nfull > 0)
			issue_block<NW32, AMODE>(p, cur);
		for (uint32_t k = 0; k < nfull; k++) {
			prio_remaining<H::DRAIN && AMODE != AMODE_A1>(nfull - k);
			const uint8_t *bp = p + (size_t)k * H::BLOCK;
			Raw<NW32> nxt;
			if (k + 1 < nfull)
				issue_block<NW32, AMODE>(bp + H::BLOCK, nxt);
			uint32_t w[NW32];
			finish_block<NW32, AMODE>(bp, cur, w);
			H::compress(st, w);
			cur = nxt;
		}
	} else {
		for (uint32_t k = 0; k < nfull; k++) {
			prio_remaining<H::DRAIN && AMODE != AMODE_A1>(nfull - k);
			const uint8_t *bp = p + (size_t)k * H::BLOCK;
			Raw<NW32> cur;
			issue_block<NW32, AMODE>(bp, cur);
			uint32_t w[NW32];
			finish_block<NW32, AMODE>(bp, cur, w);
			H::compress(st, w);
		}
	}
}

/*
 * SHA*Pad (src/sha2.c:495-543 / :784-832): the len % BLOCK tail bytes, the
 * 0x80 terminator, zero fill and the big-endian bit count `bits` (the whole
 * message, including any prefix hashed before p), in one or two blocks.
 * PADCONST: the caller knows len % BLOCK == 0 for every lane, so the pad
 * block is constant and its K[t] + W[t] schedule comes precomputed in kw.
 */
template <class H, bool PADCONST>
__device__ __forceinline__ void finish(const uint8_t *p, uint32_t len,
    uint64_t bits, const typename H::word *kw, typename H::State &st)
{
	constexpr int NW32 = H::NW32;
	if (PADCONST) {
		if (sizeof(typename H::word) == 4)
			compress256_kw<H::ASM>(*reinterpret_cast<uint32_t(*)[8]>(&st),
			    reinterpret_cast<const uint32_t *>(kw));
		else
			compress512_kw(*reinterpret_cast<uint64_t(*)[8]>(&st),
			    reinterpret_cast<const uint64_t *>(kw));
		return;
	}
	const uint32_t nfull = len / H::BLOCK;
	const uint32_t rem = len % H::BLOCK;
	uint32_t w[NW32];
	tail_block<NW32>(p + (size_t)nfull * H::BLOCK, rem, w);
	if (rem >= (uint32_t)(H::BLOCK - H::LENBYTES)) {
		/* No room for the length: this block, then a zero block. */
		H::compress(st, w);
#pragma unroll
		for (int i = 0; i < NW32; i++)
			w[i] = 0;
	}
	w[NW32 - 2] = (uint32_t)(bits >> 32);
	w[NW32 - 1] = (uint32_t)bits;
	H::compress(st, w);
}

/* Init + Update + Pad of one whole message (Final's store is the caller's). */
template <class H, int AMODE, bool PADCONST, bool PREFETCH = H::PREFETCH>
__device__ __forceinline__ void digest_one(const uint8_t *p, uint32_t len,
    int is384, const typename H::word *kw, typename H::State &st)
{
	H::init(st, is384);
	absorb<H, AMODE, PREFETCH>(p, len, st);
	finish<H, PADCONST>(p, len, (uint64_t)len << 3, kw, st);
}

/* Constant-pad schedule passed by value (kernarg -> SGPRs / LDS). */
template <class W>
struct PadKW {
	W kw[sizeof(W) == 4 ? 64 : 80];
};

/* One lane of the fixed-stride layout: packet i. */
template <class H, int AMODE, bool PADCONST, bool PREFETCH = H::PREFETCH>
__device__ __forceinline__ void fixed_lane(uint64_t i,
    const uint8_t *__restrict__ base, uint64_t stride, uint32_t len,
    uint8_t *__restrict__ out, uint32_t dlen, int is384,
    const typename H::word *kw)
{
	typename H::State st;
	digest_one<H, AMODE, PADCONST, PREFETCH>(base + i * stride, len, is384,
	    kw, st);
	uint32_t o[16];
	H::out_words(st, o, is384);
	if (dlen == 48)
		store_digest<48>(out + i * 48, o);
	else
		store_digest<H::DLEN>(out + i * H::DLEN, o);
}

/* (no occupancy request: 6 waves per SIMD asked of the fixed SHA-512
 * kernel measured -1.4 %, profiles/round2/occupancy_request_ab.txt) */
template <class H, int AMODE, bool PADCONST>
__global__ __launch_bounds__(256) void fixed_kernel(const uint8_t *__restrict__ base,
    uint64_t stride, uint32_t len, uint64_t n, uint8_t *__restrict__ out,
    uint32_t dlen, int is384, PadKW<typename H::word> pad)
{
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (sizeof(typename H::word) == 8) {
		if (PADCONST)
			k512_lds_fill_pad(pad);
		else
			k512_lds_fill();
	}
	if (i >= n)
		return;
	fixed_lane<H, AMODE, PADCONST>(i, base, stride, len, out, dlen, is384,
	    pad.kw);
}

/*
 * K[t] + W[t] of the SHA-256 pad block of every message whose length is a
 * whole number of blocks, 64 * j bytes for j < NET2_PADTAB_N (up to
 * 65,536-byte payloads plus an HMAC key block): 0x80, zero fill, bit count
 * 512 * j (SHA256Pad for usedspace == 0, src/sha2.c:520-526).  Evaluated
 * at compile time into constant memory, so a wave whose lanes all carry the
 * same such length reads its pad schedule with scalar loads instead of
 * expanding it (48 of 64 schedule words, ~480 VALU instructions per lane),
 * as fixed_kernel does with its kernel-argument copy.
 */
#define NET2_PADTAB_N 1026

struct PadTab256 {
	uint32_t kw[NET2_PADTAB_N][64];
};

constexpr uint32_t cx_ror32(uint32_t x, int n)
{
	return (x >> n) | (x << (32 - n));
}

constexpr PadTab256 make_padtab256()
{
	PadTab256 t{};
	for (int j = 0; j < NET2_PADTAB_N; j++) {
		uint32_t w[64] = {};
		const uint64_t bits = (uint64_t)j * 512;
		w[0] = 0x80000000u;
		w[14] = (uint32_t)(bits >> 32);
		w[15] = (uint32_t)bits;
		for (int r = 16; r < 64; r++) {
			const uint32_t s0 = cx_ror32(w[r - 15], 7) ^
			    cx_ror32(w[r - 15], 18) ^ (w[r - 15] >> 3);
			const uint32_t s1 = cx_ror32(w[r - 2], 17) ^
			    cx_ror32(w[r - 2], 19) ^ (w[r - 2] >> 10);
			w[r] = w[r - 16] + s0 + w[r - 7] + s1;
		}
		for (int r = 0; r < 64; r++)
			t.kw[j][r] = K256[r] + w[r];
	}
	return t;
}

__constant__ const PadTab256 g_padtab256 = make_padtab256();

/*
 * The wave-uniform pad schedule for messages of `bytes` total bytes (any
 * prefix included), or nullptr when the wave's live lanes differ in length,
 * the length is not a whole number of blocks or lies past the table.
 */
template <class H>
__device__ __forceinline__ const typename H::word *uniform_pad_kw(bool live,
    uint64_t bytes)
{
	if (sizeof(typename H::word) != 4)
		return nullptr;
	const uint32_t lo = (uint32_t)bytes;
	const uint32_t b0 = __builtin_amdgcn_readfirstlane(lo);
	if (!__all(!live || bytes == b0) || b0 % 64 != 0 ||
	    b0 / 64 >= NET2_PADTAB_N)
		return nullptr;
	return reinterpret_cast<const typename H::word *>(
	    g_padtab256.kw[b0 / 64]);
}

/*
 * The SHA-512 counterpart: K[t] + W[t] of the pad block of a 128 * j byte
 * message (0x80, zeros, 128-bit bit count 1024 * j; SHA512Pad,
 * src/sha2.c:784-832) for j < NET2_PADTAB512_N, 329 KB of constant memory.
 * SHA-512 compressions read their round constants from the workgroup's LDS
 * copy (k512_lds, sha2_device.h), so the table row is staged there, in the
 * [80, 160) half the fixed kernel's constant pad block uses; that makes the
 * choice per workgroup: every live lane of it must share the length.
 */
#define NET2_PADTAB512_N 514

struct PadTab512 {
	uint64_t kw[NET2_PADTAB512_N][80];
};

constexpr uint64_t cx_ror64(uint64_t x, int n)
{
	return (x >> n) | (x << (64 - n));
}

constexpr PadTab512 make_padtab512()
{
	PadTab512 t{};
	for (int j = 0; j < NET2_PADTAB512_N; j++) {
		uint64_t w[80] = {};
		w[0] = 0x8000000000000000ull;
		w[15] = (uint64_t)j * 1024;	/* w[14]: high half of the count */
		for (int r = 16; r < 80; r++) {
			const uint64_t s0 = cx_ror64(w[r - 15], 1) ^
			    cx_ror64(w[r - 15], 8) ^ (w[r - 15] >> 7);
			const uint64_t s1 = cx_ror64(w[r - 2], 19) ^
			    cx_ror64(w[r - 2], 61) ^ (w[r - 2] >> 6);
			w[r] = w[r - 16] + s0 + w[r - 7] + s1;
		}
		for (int r = 0; r < 80; r++)
			t.kw[j][r] = K512[r] + w[r];
	}
	return t;
}

__constant__ const PadTab512 g_padtab512 = make_padtab512();

/*
 * Workgroup-uniform whole-block length for SHA-512: stage its pad schedule
 * in k512_lds[80, 160) and return true.  Called by every thread of the
 * workgroup (it synchronises), after k512_lds_fill().
 */
__device__ __forceinline__ bool block_pad512(bool live, uint64_t bytes)
{
	__shared__ uint64_t b0s;
	if (threadIdx.x == 0)
		b0s = live ? bytes : 1;	/* thread 0 is live if any thread is */
	__syncthreads();
	const uint64_t b0 = b0s;
	const bool same = __syncthreads_and(!live || bytes == b0);
	if (!same || b0 % 128 != 0 || b0 / 128 >= NET2_PADTAB512_N)
		return false;
	for (unsigned t = threadIdx.x; t < 80; t += blockDim.x)
		k512_lds[80 + t] = g_padtab512.kw[b0 / 128][t];
	__syncthreads();
	return true;
}

/* The state as big-endian digest words (SHA*Final's byte order). */
template <class H>
__device__ __forceinline__ int digest_words(const typename H::State &st,
    int is384, uint32_t (&w)[H::NW32])
{
	if (sizeof(typename H::word) == 4) {
#pragma unroll
		for (int i = 0; i < 8; i++)
			w[i] = (uint32_t)st[i];
		return 8;
	}
#pragma unroll
	for (int i = 0; i < 8; i++) {
		w[2 * i] = hi32((uint64_t)st[i]);
		w[2 * i + 1] = lo32((uint64_t)st[i]);
	}
	return is384 ? 12 : 16;
}

/* Midstate `which` (0 inner, 1 outer) from LDS into a state. */
template <class H>
__device__ __forceinline__ void load_mid(const uint32_t (*mid)[16], int which,
    typename H::State &st)
{
	/* opaque zero: keeps the reads where they are written (not hoisted
	 * and shared across the address-mode branches) */
	uint32_t z;
	asm volatile("s_mov_b32 %0, 0" : "=s"(z));
	mid += z;
#pragma unroll
	for (int i = 0; i < 8; i++) {
		if (sizeof(typename H::word) == 4)
			st[i] = mid[which][i];
		else
			st[i] = mk64(mid[which][2 * i + 1], mid[which][2 * i]);
	}
}

/* digest_one for the variable layout: one block loop, and the pad block
 * from the constant table when the wave (SHA-256: kw) or the workgroup
 * (SHA-512: k512_lds) has one. */
template <class H, int AMODE, bool PREFETCH = H::PREFETCH>
__device__ __forceinline__ void var_digest(const uint8_t *p, uint32_t len,
    int is384, const typename H::word *kw, bool padtab, typename H::State &st)
{
	H::init(st, is384);
	absorb<H, AMODE, PREFETCH>(p, len, st);
	if (padtab)
		finish<H, true>(p, len, 0, kw, st);
	else
		finish<H, false>(p, len, (uint64_t)len << 3, nullptr, st);
}

/*
 * The visiting order a launch's binning left in ws (sha2_launch.h): perm,
 * or submission order (nullptr) when ws is NULL or when that binning launch
 * -- the one tagged `launch` -- found its global histogram inconsistent
 * (BinHdr::bad == launch, bin_onepass_kernel): its workgroups may then have
 * written a mix of binned and identity positions.  One scalar load.
 */
__device__ __forceinline__ const uint32_t *bin_perm(
    const uint32_t *__restrict__ ws, uint32_t launch)
{
	if (ws == nullptr || ws[NET2_BIN_W_BAD] == launch)
		return nullptr;
	return ws + NET2_BIN_WS_WORDS;
}

/*
 * Variable-length packets, visited in binned order: lane g hashes packet
 * perm[g] (perm == NULL: identity).  The address mode is chosen per wave:
 * if every lane's packet start is 16-byte aligned the wave takes the vector
 * load path, else the byte-aligned one.  A SHA-256 wave (SHA-512:
 * workgroup) of one whole-block length, e.g. a bin of a batch of fixed
 * sizes, takes its pad schedule from g_padtab256 (g_padtab512).
 * (No occupancy request: 5 waves asked of the variable-length SHA-256
 * kernel measured flat, of the SHA-512 one -2 %,
 * profiles/round2/occupancy_request_ab.txt.)
 */
/* One packet of var_kernel: binned position g (SHA-512: block_pad512 is a
 * workgroup barrier, so every thread calls this equally often). */
template <class H>
__device__ __forceinline__ void var_item(uint64_t g,
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offsets,
    const uint32_t *__restrict__ lens, const uint32_t *__restrict__ perm,
    uint64_t n, uint8_t *__restrict__ out, uint32_t dlen, int is384)
{
	const bool live = g < n;
	uint64_t i = live ? (perm ? (uint64_t)perm[g] : g) : 0;
	if (i >= n)	/* a corrupt workspace: never read out of bounds */
		i = g;
	const uint8_t *p = base + (live ? offsets[i] : 0);
	const uint32_t len = live ? lens[i] : 0;
	typename H::State st;
	const typename H::word *kw = uniform_pad_kw<H>(live, len);
	bool padtab = kw != nullptr;
	if constexpr (sizeof(typename H::word) == 8)
		padtab = block_pad512(live, len);

	if (OnePath<H>::value ||
	    __all((reinterpret_cast<uintptr_t>(p) & 15) == 0))
		var_digest<H, AMODE_A16>(p, len, is384, kw, padtab, st);
	else if (__all((reinterpret_cast<uintptr_t>(p) & 3) == 0))
		var_digest<H, AMODE_A4>(p, len, is384, kw, padtab, st);
	else
		/* no prefetch on the byte-aligned path: its double buffer
		 * (17 words each) set the kernel's VGPRs (105 against 96, 5
		 * waves); C3 +0.3 %, byte-aligned mix +0.7 % without,
		 * profiles/round2/var_a1_prefetch_ab.txt */
		var_digest<H, AMODE_A1, false>(p, len, is384, kw, padtab, st);
	materialize<H>(st);
	if (!live)
		return;
	uint32_t o[16];
	H::out_words(st, o, is384);
	if (dlen == 48)
		store_digest<48>(out + i * 48, o);
	else
		store_digest<H::DLEN>(out + i * H::DLEN, o);
}

/* ws: the binning workspace of this launch (NULL: submission order). */
template <class H>
__global__ __launch_bounds__(256) void var_kernel(const uint8_t *__restrict__ base,
    const uint64_t *__restrict__ offsets, const uint32_t *__restrict__ lens,
    const uint32_t *__restrict__ ws, uint32_t launch, uint64_t n,
    uint8_t *__restrict__ out, uint32_t dlen, int is384)
{
	if (sizeof(typename H::word) == 8)
		k512_lds_fill();
	var_item<H>((uint64_t)blockIdx.x * blockDim.x + threadIdx.x, base,
	    offsets, lens, bin_perm(ws, launch), n, out, dlen, is384);
}

/* ---- HMAC (RFC 2104) ------------------------------------------------------ */

/*
 * The keyed rows of the registry (HMAC-SHA256/384/512, key length = digest
 * length, cxx_src/hash-openssl.cc:417-429), i.e. the per-datagram
 * authenticator of net2_packet_encode/decode (types/packet.n2t:246,417),
 * over a whole batch under one connection key:
 *   HMAC(K, m) = H((K' ^ opad) || H((K' ^ ipad) || m)),  K' = K zero-padded.
 * The two key blocks -- the same for every packet of a launch -- are
 * compressed once on the host (hmac_midstates below) and arrive as kernel
 * arguments: the ipad / opad midstates, copied to LDS at kernel entry; every
 * lane hashes its packet from the inner midstate (bit count includes the key
 * block) and finishes with one outer compression over the inner digest.
 * (Until round 4 wave 0 of every workgroup compressed the key blocks while
 * the other waves waited: a second instance of the round code in the kernel,
 * which held the fixed-layout HMAC-SHA512 kernel at 115 VGPRs.)
 */
struct HMid {
	/* [0] K' ^ ipad, [1] K' ^ opad as digest words (SHA-256: 8 state words;
	 * SHA-384/512: hi, lo of each 64-bit word); [2..3] the same for the
	 * alternate rx key (HMAC_BURST_RX with rx.alt) */
	uint32_t w[4][16];
};

/* Inner hash from the ipad midstate, one address mode. */
template <class H, int AMODE, bool PADCONST, bool PREFETCH = H::PREFETCH>
__device__ __forceinline__ void hmac_inner(const uint8_t *p, uint32_t len,
    const uint32_t (*mid)[16], const typename H::word *kw,
    typename H::State &st, bool padtab)
{
	load_mid<H>(mid, 0, st);
	absorb<H, AMODE, PREFETCH>(p, len, st);
	if (!PADCONST && padtab)
		finish<H, true>(p, len, 0, kw, st);
	else
		finish<H, PADCONST>(p, len, ((uint64_t)len + H::BLOCK) << 3, kw,
		    st);
}

template <class H, bool PADCONST>
__device__ __forceinline__ void hmac_lane(const uint8_t *p, uint32_t len,
    int is384, int amode, const uint32_t (*mid)[16],
    const typename H::word *kw, typename H::State &st, bool padtab = false)
{
	constexpr int NW32 = H::NW32;
	/* the midstates stay in LDS and are read where they are used, so
	 * neither is held in VGPRs across the block loop */
	if (amode == AMODE_A16)
		hmac_inner<H, AMODE_A16, PADCONST>(p, len, mid, kw, st, padtab);
	else if (amode == AMODE_A4)
		hmac_inner<H, AMODE_A4, PADCONST>(p, len, mid, kw, st, padtab);
	else
		hmac_inner<H, AMODE_A1, PADCONST>(p, len, mid, kw, st, padtab);

	/* outer: one block = inner digest || 0x80 || 0... || bit count */
	uint32_t w[NW32];
#pragma unroll
	for (int i = 0; i < NW32; i++)
		w[i] = 0;
	const int dw = digest_words<H>(st, is384, w);
#pragma unroll
	for (int i = 12; i < 16; i++)		/* SHA-384 keeps 12 words */
		if (i >= dw)
			w[i] = 0;
	w[dw] = 0x80000000u;
	const uint64_t obits = (uint64_t)(H::BLOCK + 4 * dw) << 3;
	w[NW32 - 2] = (uint32_t)(obits >> 32);
	w[NW32 - 1] = (uint32_t)obits;
	load_mid<H>(mid, 1, st);
	H::compress(st, w);
}

/*
 * PADCONST: fixed layout with fixed_len % BLOCK == 0, so the inner pad
 * block (bit count = (BLOCK + fixed_len) * 8) is the same for every lane
 * and its K + W schedule comes precomputed in pad, as in fixed_kernel.
 *
 * MODE (variable layout only for SIGN / VERIFY): datagram i is
 * base[offsets[i] .. + lens[i]) = hash field (dlen bytes) || message, the
 * wire order of net2_packet_encode (the hash is prepended,
 * types/packet.n2t:417-427) and net2_packet_decode (it is removed first,
 * :236-244).
 *   HMAC_DIGESTS: digest of the whole packet to out + i * dlen;
 *   HMAC_SIGN:    digest of the message into the datagram's hash field
 *                 (out == base, writable); datagrams shorter than dlen are
 *                 left untouched;
 *   HMAC_VERIFY:  out[i] = 0 if the hash field equals the digest of the
 *                 message (the net2_buffer_cmp of :254), 1 if it does not,
 *                 2 if the datagram is shorter than dlen (:240-244).
 */
enum { HMAC_DIGESTS = 0, HMAC_SIGN = 1, HMAC_VERIFY = 2, HMAC_BURST_RX = 3,
    HMAC_BURST_TX = 4 };

/*
 * Packet-burst codes (the burst kernels below): the status byte is the
 * NET2_P{EN,DE}CODE_* code, | BURST_VERIFY when the HMAC verdict of the
 * datagram's region decides it.
 */
#define BURST_VERIFY 0x80u
#define PKT_PH_ENCRYPTED 0x00000001u	/* types/packet.n2t:27 */
#define PKT_PH_SIGNED 0x00000002u	/* types/packet.n2t:28 */
#define PKT_PH_ALTKEY 0x80000000u	/* types/packet.n2t:34 */
#define PKT_OK 0
#define PKT_RESOURCE 1
#define PKT_BAD 2
#define PKT_UNSAFE 3

__device__ __forceinline__ uint32_t load_be32_bytes(const uint8_t *p)
{
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) |
	    ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

/*
 * HMAC_BURST_RX: the per-datagram bookkeeping of net2_packet_decode folded
 * into the VERIFY kernel.  offsets / lens describe whole wire datagrams;
 * each lane decodes its datagram's header (cp_packet_header,
 * types/packet.n2t:196-198), checks the flags against the negotiated keys
 * (:217-221; a hash key is always set on this path), and, when PH_SIGNED,
 * verifies "hash field || payload" after the 8-byte header (:233-257) --
 * exactly burst_prep_kernel's RX branch followed by HMAC_VERIFY, without
 * prep's extra pass over every datagram's first line.  Writes the status
 * (| BURST_VERIFY), seq and flags per datagram and the verdict to out.
 * HMAC_BURST_TX: the same for net2_packet_encode (out == base): the lane
 * takes seq / flags from the caller's arrays, applies the encode-side flag
 * checks (:364-370) and the room check, writes the header (:384-392) and
 * signs the payload into the hash field (:410-427), as burst_prep_kernel's
 * TX branch followed by HMAC_SIGN; status per datagram.
 */
/* (struct BurstArgs: sha2_launch.h) */



/*
 * One datagram / packet of hmac_kernel: binned position g (live: g < n).
 * Shares the workgroup's key midstates (mid) and, for SHA-512, its LDS
 * constant table; calls block_pad512 (a workgroup barrier), so every
 * thread of the workgroup calls it the same number of times.  IS384 and
 * the digest length are compile-time constants of the kernel instance
 * (SHA-384 is its own instance: the outer block's 0x80 word and zero fill
 * fold into its schedule).
 */
template <class H, bool PADCONST, int MODE, bool IS384>
__device__ __forceinline__ void hmac_item(uint64_t g,
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offsets,
    const uint32_t *__restrict__ lens, const uint32_t *__restrict__ perm,
    uint64_t stride, uint32_t fixed_len, uint64_t n,
    uint8_t *__restrict__ out, const PadKW<typename H::word> &pad,
    const BurstArgs &rx, const uint32_t (*mid)[16])
{
	constexpr int is384 = IS384;
	constexpr uint32_t dlen = sizeof(typename H::word) == 4 ? 32 :
	    IS384 ? 48 : 64;
	const uint32_t (*lmid)[16] = mid;	/* this lane's key */
	const bool live = g < n;
	uint64_t i = g;
	const uint8_t *p;
	uint32_t len;
	if (offsets != nullptr) {
		i = live ? (perm ? (uint64_t)perm[g] : g) : 0;
		if (i >= n)	/* a corrupt workspace: never out of bounds */
			i = g;
		p = base + (live ? offsets[i] : 0);
		len = live ? lens[i] : 0;
	} else {
		p = base + (live ? i * stride : 0);
		len = live ? fixed_len : 0;
	}
	uint32_t rx_st = PKT_OK, rx_seq = 0, rx_fl = 0;
	/* TX with rx.rec (the host path): instead of sealing in place, every
	 * live lane fills the record of its binned position g -- hash field at
	 * +0, then header, datagram index and code -- so a wave's stores cover
	 * one contiguous stretch of (host) memory; the address is formed where
	 * it is used, not held across the hash */
	if (MODE == HMAC_BURST_TX) {
		if (live) {
			rx_seq = rx.seq[i];
			rx_fl = rx.flags[i];
		}
		const bool sg = (rx_fl & PKT_PH_SIGNED) != 0;
		const bool cr = (rx_fl & PKT_PH_ENCRYPTED) != 0;
		if (!sg || cr != (rx.enc_set != 0))
			rx_st = PKT_UNSAFE;
		else if (len < 8 + dlen)
			rx_st = PKT_RESOURCE;	/* no room for header and hash */
		const bool ok = live && rx_st == PKT_OK;
		if (live && rx.rec != nullptr) {
			*reinterpret_cast<uint4 *>(rx.rec + g * (dlen + 16) + dlen) =
			    make_uint4(ok ? bswap32(rx_seq) : 0u,
			    ok ? bswap32(rx_fl) : 0u, (uint32_t)i, rx_st);
		} else if (ok) {
			uint8_t *h = out + (p - base);
#pragma unroll
			for (int b = 0; b < 4; b++) {
				h[b] = (uint8_t)(rx_seq >> (24 - 8 * b));
				h[4 + b] = (uint8_t)(rx_fl >> (24 - 8 * b));
			}
		}
		if (ok) {
			p += 8;
			len -= 8;
		} else {
			len = 0;
		}
		if (live && rx.rec == nullptr)
			rx.status[i] = (uint8_t)rx_st;
	}
	if (MODE == HMAC_BURST_RX) {
		if (len < 8) {
			rx_st = PKT_BAD;	/* header decode fails */
		} else {
			rx_seq = load_be32_bytes(p);
			rx_fl = load_be32_bytes(p + 4);
		}
		/* net2_ck_rx_key (src/conn_keys.c:447-476): the alternate key
		 * when the datagram says so or lies past the cutoff */
		const bool use_alt = rx_st == PKT_OK && rx.alt &&
		    ((rx_fl & PKT_PH_ALTKEY) != 0 || (!rx.no_cutoff &&
		    rx_seq - rx.rx_start >= rx.cutoff - rx.rx_start));
		if (use_alt)
			lmid = mid + 2;
		const int enc_set = use_alt ? rx.alt_enc_set : rx.enc_set;
		if (rx_st == PKT_OK && ((rx_fl & PKT_PH_SIGNED) == 0 ||
		    (enc_set && (rx_fl & PKT_PH_ENCRYPTED) == 0)))
			rx_st = PKT_UNSAFE;
		if (rx_st == PKT_OK) {
			rx_st |= BURST_VERIFY;	/* hash field || payload */
			p += 8;
			len -= 8;
		} else {
			len = 0;
		}
		/* stored now, so none of them is held across the hash */
		if (live) {
			rx.status[i] = (uint8_t)rx_st;
			rx.seq[i] = rx_seq;
			rx.flags[i] = rx_fl;
		}
	}
	const bool short_dgram = MODE != HMAC_DIGESTS && len < dlen;
	if (MODE != HMAC_DIGESTS) {
		p += short_dgram ? 0 : dlen;
		len = short_dgram ? 0 : len - dlen;
	}
	typename H::State st;
	const uintptr_t pa = reinterpret_cast<uintptr_t>(p);
	const int amode = OnePath<H>::value || __all((pa & 15) == 0) ? AMODE_A16 :
	    __all((pa & 3) == 0) ? AMODE_A4 : AMODE_A1;
	/* a variable-layout SHA-256 wave of one whole-block inner length (key
	 * block included) takes its inner pad schedule from g_padtab256 */
	const typename H::word *kw = nullptr;
	bool padtab = false;
	if constexpr (!PADCONST && sizeof(typename H::word) == 4) {
		if (offsets != nullptr)
			kw = uniform_pad_kw<H>(live, (uint64_t)len + H::BLOCK);
		padtab = kw != nullptr;
	}
	/* (SHA-512: no pad table.  The workgroup-uniform g_padtab512 row the
	 * variable-length digest kernel stages costs these kernels 11 VGPRs --
	 * 106-107 against 95-96, four waves per SIMD instead of five -- and
	 * pays only when a whole workgroup's inner lengths are one multiple of
	 * 128 bytes, which no MTU mix has: payload + 128-byte key block of
	 * {64, 512, 1428 / 1500} B.) */
	hmac_lane<H, PADCONST>(p, len, is384, amode, lmid,
	    kw != nullptr ? kw : pad.kw, st, padtab);
	materialize<H>(st);
	if (!live)
		return;
	uint32_t o[16];
	H::out_words(st, o, is384);
	/* SIGN / VERIFY: the hash field, found again from the descriptor
	 * rather than held in two VGPRs across the hash: the datagram's start,
	 * past the header in the burst modes.  Its line has mostly left L2 by
	 * now (burst RX reads ~115 B more per datagram than round 4,
	 * profiles/pmc_burst_rx.json): HBM bytes, no time on this VALU-bound
	 * kernel */
	const uint8_t *field = MODE == HMAC_DIGESTS ? nullptr :
	    base + offsets[i] + (MODE == HMAC_BURST_RX || MODE == HMAC_BURST_TX ?
	    8 : 0);
	if (MODE == HMAC_VERIFY || MODE == HMAC_BURST_RX) {
		/* o[] holds the digest bytes little-endian per word, the order
		 * store_digest writes them in */
		uint32_t diff = 0;
		constexpr int NO = dlen / 4;
		if (!short_dgram && amode == AMODE_A16) {
			/* field = message start - dlen: 16-byte aligned as well
			 * (SHA-512: the one address path reads it at any alignment);
			 * all loads issued at once (a per-byte loop waited out one
			 * memory latency per byte) */
			const u32x4 *f = reinterpret_cast<const u32x4 *>(field);
#pragma unroll
			for (int k = 0; k < NO / 4; k++) {
				const u32x4 v = f[k];
				diff |= (v.x ^ o[4 * k]) | (v.y ^ o[4 * k + 1]) |
				    (v.z ^ o[4 * k + 2]) | (v.w ^ o[4 * k + 3]);
			}
		} else if (!short_dgram && amode == AMODE_A4) {
			const uint32_t *f = reinterpret_cast<const uint32_t *>(field);
#pragma unroll
			for (int k = 0; k < NO; k++)
				diff |= f[k] ^ o[k];
		} else if (!short_dgram) {
#pragma unroll
			for (int j = 0; j < (int)dlen; j++)
				diff |= field[j] ^
				    ((o[j >> 2] >> (8 * (j & 3))) & 0xffu);
		}
		out[i] = short_dgram ? 2 : diff != 0;
		return;
	}
	constexpr bool SIGNS = MODE == HMAC_SIGN || MODE == HMAC_BURST_TX;
	if (SIGNS && short_dgram)
		return;
	if (MODE == HMAC_BURST_TX && rx.rec != nullptr)
		store_digest<dlen>(rx.rec + g * (dlen + 16), o);
	else
		store_digest<dlen>(SIGNS ? out + (field - base) : out + i * dlen,
		    o);
}

/*
 * ws: the binning workspace of this launch (variable layout; NULL:
 * submission order); hm: the key's midstates (HMid).  No occupancy request:
 * 5 waves asked of the SHA-512 kernels measured +3-4 % on the digests only
 * while they spilled, and -2 to -15 % on the sign / verify / burst modes
 * (round 2, profiles/round2/hmac512_waves_ab.txt); the VGPR count decides.
 */
template <class H, bool PADCONST, int MODE, bool IS384>
__global__ __launch_bounds__(256) void hmac_kernel(const uint8_t *__restrict__ base,
    const uint64_t *__restrict__ offsets, const uint32_t *__restrict__ lens,
    const uint32_t *__restrict__ ws, uint32_t launch, uint64_t stride,
    uint32_t fixed_len, uint64_t n, uint8_t *__restrict__ out, HMid hm,
    PadKW<typename H::word> pad, BurstArgs rx)
{
	/* [0..1]: the key's ipad / opad midstates; [2..3]: the alternate rx
	 * key's (HMAC_BURST_RX with rx.alt) */
	__shared__ uint32_t mid[4][16];
	const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	/* one lane copies them (the by-value argument read with constant
	 * indices only: a dynamic index would copy it to scratch) */
	if (threadIdx.x == 0) {
		constexpr int NK = MODE == HMAC_BURST_RX ? 4 : 2;
		/* whole chaining values (SHA-384's too) */
		constexpr int NWD = sizeof(typename H::word) == 4 ? 8 : 16;
#pragma unroll
		for (int k = 0; k < NK; k++)
#pragma unroll
			for (int j = 0; j < NWD; j++)
				mid[k][j] = hm.w[k][j];
	}
	if (sizeof(typename H::word) == 8) {
		/* (both synchronise the workgroup) */
		if (PADCONST)
			k512_lds_fill_pad(pad);
		else
			k512_lds_fill();
	} else {
		__syncthreads();
	}
	hmac_item<H, PADCONST, MODE, IS384>(g, base, offsets, lens,
	    offsets != nullptr ? bin_perm(ws, launch) : nullptr, stride,
	    fixed_len, n, out, pad, rx, mid);
}

/* ---- coalesced small jobs (sha2_coalesce.cpp) ------------------------------- */

/*
 * One lane = one request of the single-message entry points
 * (net2_hashctx_hashiov, the SHA2_CTX streaming calls, net2_ph_to_iv), which
 * the reference runs one payload at a time on threadpool workers
 * (types/signature.n2t:92,147, src/sign.c:298-307, types/packet.n2t:134-142).
 * Concurrent requests are gathered by the host into one staging buffer,
 * every message already padded to whole blocks (SHA*Pad's layout, or the
 * K' ^ ipad block ahead of it for HMAC), so a lane only compresses.
 */
template <class H>
__global__ __launch_bounds__(64) void job_kernel(const uint8_t *__restrict__ stage,
    const Net2Job *__restrict__ jobs, uint32_t n, uint8_t *__restrict__ out,
    uint32_t *done, uint32_t chunk)
{
	constexpr int NW32 = H::NW32;
	typedef typename H::word W;
	if (sizeof(W) == 8)
		k512_lds_fill();
	const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
	if (j >= n)
		return;
	const Net2Job jb = jobs[j];
	const int is384 = (jb.flags & 0xffu) == NET2_ALG_SHA384;
	typename H::State st;
	if (jb.flags & NET2_JOB_STATE) {
		const W *s0 = reinterpret_cast<const W *>(stage + jb.aux);
#pragma unroll
		for (int i = 0; i < 8; i++)
			st[i] = s0[i];
	} else {
		H::init(st, is384);
	}
	/* absorb takes a 32-bit length: a job of 4 GiB or more (nblk up to
	 * UINT32_MAX blocks) goes through in chunks of whole blocks (chunk: a
	 * multiple of 128 below 4 GiB, 2 GiB unless a test asks for less) */
	{
		const uint8_t *q = stage + jb.data;
		uint64_t left = (uint64_t)jb.nblk * H::BLOCK;
		while (left > chunk) {
			absorb<H, AMODE_A16>(q, chunk, st);
			q += chunk;
			left -= chunk;
		}
		absorb<H, AMODE_A16>(q, (uint32_t)left, st);
	}
	if (jb.flags & NET2_JOB_HMAC) {
		/* outer hash: IV, K' ^ opad, inner digest || 0x80 || bit count */
		uint32_t w[NW32];
#pragma unroll
		for (int i = 0; i < NW32; i++)
			w[i] = 0;
		const int dw = digest_words<H>(st, is384, w);
#pragma unroll
		for (int i = 12; i < 16; i++)		/* SHA-384 keeps 12 words */
			if (i >= dw)
				w[i] = 0;
		w[dw] = 0x80000000u;
		const uint64_t obits = (uint64_t)(H::BLOCK + 4 * dw) << 3;
		w[NW32 - 2] = (uint32_t)(obits >> 32);
		w[NW32 - 1] = (uint32_t)obits;
		H::init(st, is384);
		Raw<NW32> r;
		issue_block<NW32, AMODE_A16>(stage + jb.aux, r);
		uint32_t kb[NW32];
		finish_block<NW32, AMODE_A16>(stage + jb.aux, r, kb);
		H::compress(st, kb);
		H::compress(st, w);
	}
	W *o = reinterpret_cast<W *>(out + 64 * (size_t)j);
#pragma unroll
	for (int i = 0; i < 8; i++)
		o[i] = st[i];
	/* count the wave in once all of its lanes' results are visible to the
	 * host (the workgroup is one wave; lane 0 is always live) */
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
	if (threadIdx.x == 0)
		__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELEASE,
		    __HIP_MEMORY_SCOPE_SYSTEM);
}

/*
 * Latency form of job_kernel: one wave per job, for batches small enough
 * that the GPU is otherwise idle (a lone caller, a few threads).  A lane of
 * job_kernel runs message expansion and rounds of every block one after the
 * other; here the 64 lanes first expand up to 64 blocks of the job at once
 * (block b's K[t] + W[t] by lane b, into LDS -- the schedule of a block
 * depends only on its message words, not on the chaining state), then the
 * wave runs only the rounds, block after block, reading K + W from LDS.
 * About a third of a compression's instructions leave the serial chain.
 */
#define NET2_JOB_ROW256 65	/* dwords per LDS row: odd, so the 64 lanes'
				 * row writes fall in distinct banks */
#define NET2_JOB_ROW512 81	/* qwords per row */

template <int T>
struct Sched256 {
	__device__ __forceinline__ static void run(uint32_t (&w)[16],
	    uint32_t *row)
	{
		const uint32_t wt = T < 16 ? w[T & 15] : expand256<T, false>(w);
		row[T] = wt + K256[T];
		Sched256<T + 1>::run(w, row);
	}
};
template <>
struct Sched256<64> {
	__device__ __forceinline__ static void run(uint32_t (&)[16], uint32_t *) {}
};

template <int T>
struct Sched512 {
	__device__ __forceinline__ static void run(uint64_t (&w)[16],
	    uint64_t *row, const lds_k64 *kb)
	{
		const uint64_t wt = T < 16 ? w[T & 15] : expand512<T>(w);
		row[T] = addk512<T>(wt, kb);
		Sched512<T + 1>::run(w, row, kb);
	}
};
template <>
struct Sched512<80> {
	__device__ __forceinline__ static void run(uint64_t (&)[16], uint64_t *,
	    const lds_k64 *) {}
};

template <int T>
struct RowRounds512 {
	__device__ __forceinline__ static void run(uint64_t (&s)[8],
	    const uint64_t *row)
	{
		round512<T>(s, row[T]);
		RowRounds512<T + 1>::run(s, row);
	}
};
template <>
struct RowRounds512<80> {
	__device__ __forceinline__ static void run(uint64_t (&)[8],
	    const uint64_t *) {}
};

/* Expand block `blk` (big-endian words) into its K + W row. */
template <class H>
__device__ __forceinline__ void sched_row(uint32_t (&blk)[H::NW32],
    typename H::word *row)
{
	if constexpr (sizeof(typename H::word) == 4) {
		Sched256<0>::run(blk, row);
	} else {
		uint64_t w[16];
#pragma unroll
		for (int i = 0; i < 16; i++)
			w[i] = mk64(blk[2 * i + 1], blk[2 * i]);
		Sched512<0>::run(w, row, k512_base());
	}
}

/* The rounds of one block from its K + W row (all lanes, same state). */
template <class H>
__device__ __forceinline__ void rounds_row(typename H::State &st,
    const typename H::word *row)
{
	if constexpr (sizeof(typename H::word) == 4) {
		compress256_kw<H::ASM>(st, row);
	} else {
		uint64_t s[8];
#pragma unroll
		for (int i = 0; i < 8; i++)
			s[i] = st[i];
		RowRounds512<0>::run(s, row);
#pragma unroll
		for (int i = 0; i < 8; i++)
			st[i] += s[i];
	}
}

template <class H>
__global__ __launch_bounds__(64) void job_wave_kernel(const uint8_t *__restrict__ stage,
    const Net2Job *__restrict__ jobs, uint8_t *__restrict__ out,
    uint32_t *done)
{
	constexpr int NW32 = H::NW32;
	typedef typename H::word W;
	constexpr int ROW = sizeof(W) == 4 ? NET2_JOB_ROW256 : NET2_JOB_ROW512;
	__shared__ W rows[64 * ROW];
	if (sizeof(W) == 8)
		k512_lds_fill();
	const uint32_t lane = threadIdx.x;
	const Net2Job jb = jobs[blockIdx.x];
	const int is384 = (jb.flags & 0xffu) == NET2_ALG_SHA384;
	typename H::State st;
	if (jb.flags & NET2_JOB_STATE) {
		const W *s0 = reinterpret_cast<const W *>(stage + jb.aux);
#pragma unroll
		for (int i = 0; i < 8; i++)
			st[i] = s0[i];
	} else {
		H::init(st, is384);
	}
	const uint8_t *p = stage + jb.data;
	for (uint32_t c0 = 0; c0 < jb.nblk; c0 += 64) {
		const uint32_t nb = min(64u, jb.nblk - c0);
		if (lane < nb) {
			const uint8_t *bp = p + (size_t)(c0 + lane) * H::BLOCK;
			Raw<NW32> r;
			issue_block<NW32, AMODE_A16>(bp, r);
			uint32_t w[NW32];
			finish_block<NW32, AMODE_A16>(bp, r, w);
			sched_row<H>(w, rows + lane * ROW);
		}
		__syncthreads();
		for (uint32_t b = 0; b < nb; b++)
			rounds_row<H>(st, rows + b * ROW);
		__syncthreads();
	}
	if (jb.flags & NET2_JOB_HMAC) {
		uint32_t w[NW32];
#pragma unroll
		for (int i = 0; i < NW32; i++)
			w[i] = 0;
		const int dw = digest_words<H>(st, is384, w);
#pragma unroll
		for (int i = 12; i < 16; i++)
			if (i >= dw)
				w[i] = 0;
		w[dw] = 0x80000000u;
		const uint64_t obits = (uint64_t)(H::BLOCK + 4 * dw) << 3;
		w[NW32 - 2] = (uint32_t)(obits >> 32);
		w[NW32 - 1] = (uint32_t)obits;
		H::init(st, is384);
		Raw<NW32> r;
		issue_block<NW32, AMODE_A16>(stage + jb.aux, r);
		uint32_t kb[NW32];
		finish_block<NW32, AMODE_A16>(stage + jb.aux, r, kb);
		H::compress(st, kb);
		H::compress(st, w);
	}
	if (lane == 0) {
		W *o = reinterpret_cast<W *>(out + 64 * (size_t)blockIdx.x);
#pragma unroll
		for (int i = 0; i < 8; i++)
			o[i] = st[i];
	}
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
	if (lane == 0)
		__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELEASE,
		    __HIP_MEMORY_SCOPE_SYSTEM);
}

/* ---- packet-header IV derivation (types/packet.n2t:100-158) ---------------- */

/*
 * iv = first ivlen bytes of D0 || D1 with D0 = SHA-256(ph), D1 = SHA-256(ph
 * || D0), ph = be32(seq) || be32(flags) (cp_packet_header,
 * packet.n2t:89-95).  The reference loops until the IV is long enough;
 * ivlen <= 64 covers two rounds, each a single block (8 + 32 bytes < 56).
 */
/* The IV of one header into out[0 .. ivlen) (ivlen <= 64). */
__device__ __forceinline__ void ph_iv_one(uint32_t s, uint32_t f,
    uint32_t ivlen, uint8_t *o)
{
	uint32_t d[16];
	uint32_t st[8], w[16];
#pragma unroll
	for (int r = 0; r < 2; r++) {
		if (r == 1 && ivlen <= 32)
			break;
#pragma unroll
		for (int j = 0; j < 16; j++)
			w[j] = 0;
		w[0] = s;
		w[1] = f;
		if (r == 0) {
			w[2] = 0x80000000u;
			w[15] = 8 * 8;
		} else {
#pragma unroll
			for (int j = 0; j < 8; j++)
				w[2 + j] = d[j];
			w[10] = 0x80000000u;
			w[15] = 40 * 8;
		}
#pragma unroll
		for (int j = 0; j < 8; j++)
			st[j] = IV256[j];
		compress256(st, w);
#pragma unroll
		for (int j = 0; j < 8; j++)
			d[8 * r + j] = st[j];
	}
	/* 16-byte stores when the IV is whole 16-byte pieces at an aligned
	 * address (AES's 16-byte IV in an n x 16 array), bytes otherwise */
	if ((ivlen & 15) == 0 && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
		uint4 *q = reinterpret_cast<uint4 *>(o);
#pragma unroll
		for (int k = 0; k < 4; k++)
			if (16u * k < ivlen)
				q[k] = make_uint4(bswap32(d[4 * k]),
				    bswap32(d[4 * k + 1]), bswap32(d[4 * k + 2]),
				    bswap32(d[4 * k + 3]));
		return;
	}
	for (uint32_t b = 0; b < ivlen; b++)
		o[b] = (uint8_t)(d[b >> 2] >> (24 - 8 * (b & 3)));
}

__global__ __launch_bounds__(256) void ph_iv_kernel(const uint32_t *__restrict__ seq,
    const uint32_t *__restrict__ flags, uint64_t n, uint32_t ivlen,
    uint8_t *__restrict__ out)
{
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	ph_iv_one(seq[i], flags[i], ivlen, out + i * ivlen);
}

/* ---- packet bursts: the hash steps of net2_packet_encode / decode ---------- */

/*
 * A datagram on the wire is the packet header (uint32 seq, uint32 flags,
 * big-endian: cp_packet_header, types/packet.n2t:89-97), then -- when
 * PH_SIGNED -- the HMAC of the rest (prepended last by net2_packet_encode,
 * :417-426, removed first by net2_packet_decode, :233-243), then the
 * payload (encrypted when PH_ENCRYPTED).  burst_prep_kernel does the
 * per-datagram bookkeeping of those functions for a whole burst and points
 * the HMAC kernel at each datagram's "hash field || payload" region;
 * burst_final_kernel folds the HMAC verdicts in and derives the IVs.
 *
 * status byte: the NET2_P{EN,DE}CODE_* code, | BURST_VERIFY when the HMAC
 * verdict of the region decides it.
 */
/* (BURST_VERIFY, the PKT_* codes and load_be32_bytes: above hmac_kernel) */

__global__ __launch_bounds__(256) void burst_prep_kernel(uint8_t *__restrict__ base,
    const uint64_t *__restrict__ offsets, const uint32_t *__restrict__ lens,
    uint64_t n, int encode, int hash_set, int enc_set, uint32_t hashlen,
    const uint32_t *__restrict__ seq_in, const uint32_t *__restrict__ flags_in,
    uint32_t *__restrict__ seq_out, uint32_t *__restrict__ flags_out,
    uint64_t *__restrict__ sub_off, uint32_t *__restrict__ sub_len,
    uint8_t *__restrict__ status)
{
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	const uint64_t off = offsets[i];
	const uint32_t len = lens[i];
	uint8_t *p = base + off;
	uint32_t seq, fl, st = PKT_OK, sl = 0;
	if (encode) {
		seq = seq_in[i];
		fl = flags_in[i];
	} else if (len < 8) {		/* cp_packet_header decode fails, :196-198 */
		seq = fl = 0;
		st = PKT_BAD;
	} else {
		seq = load_be32_bytes(p);
		fl = load_be32_bytes(p + 4);
	}
	const bool do_sign = (fl & PKT_PH_SIGNED) != 0;
	const bool do_cryp = (fl & PKT_PH_ENCRYPTED) != 0;
	if (st == PKT_OK) {
		/* flags against the negotiated keys: decode :217-221, encode
		 * :364-370 (which also refuses a flag without its key) */
		if ((!do_sign && hash_set) || (!do_cryp && enc_set) ||
		    (encode && ((do_sign && !hash_set) || (do_cryp && !enc_set))))
			st = PKT_UNSAFE;
	}
	if (st == PKT_OK && encode) {
		if (len < 8 + (do_sign ? hashlen : 0)) {
			st = PKT_RESOURCE;	/* the slot has no room for them */
		} else {
			for (int b = 0; b < 4; b++) {
				p[b] = (uint8_t)(seq >> (24 - 8 * b));
				p[4 + b] = (uint8_t)(fl >> (24 - 8 * b));
			}
			if (do_sign)
				sl = len - 8;	/* hash field || payload */
		}
	} else if (st == PKT_OK && do_sign && hash_set) {
		sl = len - 8;		/* supplied hash || payload, :233-257 */
		st |= BURST_VERIFY;
	}
	/* an empty region stays inside the datagram (a runt at the end of the
	 * buffer has no bytes at off + 8) */
	sub_off[i] = sl != 0 ? off + 8 : off;
	sub_len[i] = sl;
	status[i] = (uint8_t)st;
	if (seq_out != nullptr) {
		seq_out[i] = seq;
		flags_out[i] = fl;
	}
}

__global__ __launch_bounds__(256) void burst_final_kernel(uint64_t n,
    const uint8_t *__restrict__ status, const uint8_t *__restrict__ verdict,
    const uint32_t *__restrict__ seq, const uint32_t *__restrict__ flags,
    uint32_t ivlen, uint8_t *__restrict__ iv, uint8_t *__restrict__ result,
    uint32_t *__restrict__ seq_out, uint32_t *__restrict__ flags_out)
{
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	if (seq_out != nullptr) {	/* the decoded header, to the host */
		seq_out[i] = seq[i];
		flags_out[i] = flags[i];
	}
	uint32_t st = status[i];
	if (st & BURST_VERIFY)		/* net2_buffer_cmp, :253-257 */
		st = verdict[i] == 0 ? PKT_OK : PKT_BAD;
	/* an encrypted datagram's IV from its header, :263-279 */
	if (st == PKT_OK && iv != nullptr && ivlen > 0 &&
	    (flags[i] & PKT_PH_ENCRYPTED))
		ph_iv_one(seq[i], flags[i], ivlen, iv + i * ivlen);
	result[i] = (uint8_t)st;
}

/* ---- small bursts: a few datagrams per workgroup ------------------------- */

/*
 * Latency form of the keyed burst modes (HMAC_BURST_RX / HMAC_BURST_TX of
 * hmac_kernel, plus burst_final_kernel's fold and IV), for bursts of at most
 * BW_GMAX datagrams per SIMD.  A burst that small has at most one wave per
 * SIMD in the lane form too, so its time is one datagram's serial chain of
 * compressions, schedule expansion included (~100 us for a 1,500-byte
 * HMAC-SHA512 datagram, profiles/round6/burst_sizes_*.jsonl).  Here a
 * workgroup of two waves takes G datagrams (G <= BW_GMAX, chosen by the
 *   launcher so that the grid is about one workgroup per SIMD):
 *   wave 0 -- lane l runs datagram (l mod G)'s HMAC, so every datagram's
 *     rounds run on 64 / G lanes in lockstep and no lane idles: rounds on
 *     one lane of a wave (an EXEC mask of one) ran 27 % slower per wave and,
 *     with four workgroups per CU, twice as slow (profiles/round6/bwp_*:
 *     89 / 176 us at 64 / 1,024 datagrams against 70 / 74).  Each pass, the
 *     wave's lanes first expand K = BW_ROWS / G blocks of every one of the G
 *     messages at once (row r: datagram r / K, block c0 + r % K, loaded,
 *     padded and expanded into its K + W row in LDS -- a block's schedule
 *     depends only on its own words), then every lane runs the rounds of
 *     its datagram's K blocks from LDS; lane d < G stores datagram d.  A pass costs one row's expansion however many rows
 *     it fills, so the schedule work leaves the serial chain: a 12-block
 *     datagram takes one pass at G <= 4, five at G = 16, against twelve
 *     expansions in the lane form.  Then the outer block, the verdict (RX)
 *     or the hash field (TX), and every store of the datagram;
 *   wave 1 -- RX: lane d derives datagram d's IV from its header (two
 *     SHA-256 compressions, ph_iv_one) into LDS meanwhile, off the chain.
 * Codes, decoded headers, IVs and sealed fields are those of hmac_item +
 * burst_final_kernel (RX) / hmac_item (TX), bit for bit; the datagrams of a
 * workgroup are consecutive (no binning: the burst's time is its longest
 * datagram's either way).
 *
 * rx: RX -- seq / flags receive the decoded header (NULL: not stored);
 * TX -- seq / flags are the inputs, rec as in BurstArgs (the host path) or
 * NULL (header and hash field written into out == base).  result: the final
 * code per datagram (RX; TX without rec).
 */
#define BW_ROWS 48	/* K + W rows of LDS per workgroup (31 KB at SHA-512:
			 * four workgroups per CU; 16 rows measured no faster,
			 * profiles/round6/bw_w2r16_*.jsonl) */
#define BW_GMAX 16	/* datagrams per workgroup at most: at G = 32 a pass
			 * expands one block per datagram, the lane form's cost */

/* Block k of an inner message of mlen bytes at m (nfull whole blocks, rem
 * tail bytes, nb blocks, bit count `bits` incl. the key block) as
 * big-endian words. */
template <class H>
__device__ __forceinline__ void bw_block(const uint8_t *m, uint32_t k,
    uint32_t nfull, uint32_t rem, uint32_t nb, uint64_t bits,
    uint32_t (&w)[H::NW32])
{
	constexpr int NW32 = H::NW32;
	if (k < nfull) {
		const uint8_t *bp = m + (size_t)k * H::BLOCK;
		Raw<NW32> r;
		issue_block<NW32, AMODE_A1>(bp, r);
		finish_block<NW32, AMODE_A1>(bp, r, w);
		return;
	}
	if (k == nfull) {
		tail_block<NW32>(m + (size_t)nfull * H::BLOCK, rem, w);
	} else {
#pragma unroll
		for (int i = 0; i < NW32; i++)
			w[i] = 0;
	}
	if (k == nb - 1) {
		w[NW32 - 2] = (uint32_t)(bits >> 32);
		w[NW32 - 1] = (uint32_t)bits;
	}
}

/* LDS written by some lanes of a wave, read by others of the same wave. */
__device__ __forceinline__ void wave_lds_sync()
{
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

/* One datagram's header, key choice and the region its HMAC covers. */
struct BwDgram {
	uint32_t st, seq, fl;
	bool ok, hashed, alt;
	uint64_t off;		/* datagram start */
	uint32_t mlen;		/* message bytes after header and hash field */
};

template <int MODE, uint32_t DLEN>
__device__ __forceinline__ BwDgram bw_decode(const uint8_t *__restrict__ base,
    const uint64_t *__restrict__ offsets, const uint32_t *__restrict__ lens,
    uint64_t i, const BurstArgs &rx)
{
	BwDgram g;
	g.off = offsets[i];
	const uint32_t len = lens[i];
	const uint8_t *p = base + g.off;
	g.st = PKT_OK;
	g.seq = g.fl = 0;
	g.alt = false;
	if (MODE == HMAC_BURST_TX) {
		g.seq = rx.seq[i];
		g.fl = rx.flags[i];
		const bool sg = (g.fl & PKT_PH_SIGNED) != 0;
		const bool cr = (g.fl & PKT_PH_ENCRYPTED) != 0;
		if (!sg || cr != (rx.enc_set != 0))
			g.st = PKT_UNSAFE;
		else if (len < 8 + DLEN)
			g.st = PKT_RESOURCE;	/* no room for header and hash */
	} else {
		if (len < 8) {
			g.st = PKT_BAD;		/* header decode fails */
		} else {
			g.seq = load_be32_bytes(p);
			g.fl = load_be32_bytes(p + 4);
		}
		/* net2_ck_rx_key (src/conn_keys.c:447-476) */
		g.alt = g.st == PKT_OK && rx.alt &&
		    ((g.fl & PKT_PH_ALTKEY) != 0 || (!rx.no_cutoff &&
		    g.seq - rx.rx_start >= rx.cutoff - rx.rx_start));
		const int enc_set = g.alt ? rx.alt_enc_set : rx.enc_set;
		if (g.st == PKT_OK && ((g.fl & PKT_PH_SIGNED) == 0 ||
		    (enc_set && (g.fl & PKT_PH_ENCRYPTED) == 0)))
			g.st = PKT_UNSAFE;
	}
	g.ok = g.st == PKT_OK;
	/* after the header: hash field, then message */
	const uint32_t rlen = g.ok ? len - 8 : 0;
	g.hashed = g.ok && rlen >= DLEN;
	g.mlen = g.hashed ? rlen - DLEN : 0;
	return g;
}

template <class H, int MODE, bool IS384>
__global__ __launch_bounds__(128) void burst_wave_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offsets,
    const uint32_t *__restrict__ lens, uint64_t n, uint32_t G, HMid hm,
    BurstArgs rx, uint8_t *__restrict__ result, uint8_t *__restrict__ iv,
    uint32_t ivlen, uint8_t *__restrict__ out)
{
	constexpr int NW32 = H::NW32;
	typedef typename H::word W;
	constexpr int ROW = sizeof(W) == 4 ? NET2_JOB_ROW256 : NET2_JOB_ROW512;
	constexpr uint32_t dlen = sizeof(W) == 4 ? 32 : IS384 ? 48 : 64;
	__shared__ W rows[BW_ROWS * ROW];
	__shared__ uint32_t mid[4][16];
	__shared__ uint32_t ivw[BW_GMAX][16];
	__shared__ uint64_t geo_m[BW_GMAX];	/* message start (offset) */
	__shared__ uint32_t geo_len[BW_GMAX], geo_nb[BW_GMAX];
	if (threadIdx.x == 0) {
		constexpr int NK = MODE == HMAC_BURST_RX ? 4 : 2;
		constexpr int NWD = sizeof(W) == 4 ? 8 : 16;
#pragma unroll
		for (int k = 0; k < NK; k++)
#pragma unroll
			for (int j = 0; j < NWD; j++)
				mid[k][j] = hm.w[k][j];
	}
	if (sizeof(W) == 8)
		k512_lds_fill();	/* (synchronises the workgroup) */
	else
		__syncthreads();
	const uint32_t lane = threadIdx.x & 63;
	const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	/* every lane of a wave works on datagram slot lane % G (the G slots
	 * replicated across the wave: rounds on one lane of a wave run slower
	 * than on all of them); lane d < G owns slot d's stores */
	const uint32_t dl = lane % G;
	const uint64_t i = (uint64_t)blockIdx.x * G + dl;
	const bool live = i < n;
	const bool mine = lane < G && live;	/* this lane stores datagram i */
	BwDgram g = {};
	if (live)
		g = bw_decode<MODE, dlen>(base, offsets, lens, i, rx);

	if (wv == 1) {
		/* RX: the IV of an encrypted datagram that may verify */
		if (MODE == HMAC_BURST_RX && mine && g.ok && ivlen > 0 &&
		    iv != nullptr && (g.fl & PKT_PH_ENCRYPTED))
			ph_iv_one(g.seq, g.fl, ivlen,
			    reinterpret_cast<uint8_t *>(ivw[lane]));
		__syncthreads();
		return;
	}

	/* wave 0: HMAC of every owned message from its ipad midstate (a
	 * datagram already refused, or without room for its hash field,
	 * hashes nothing) */
	const uint32_t nfull = g.mlen / H::BLOCK;
	const uint32_t rem = g.mlen % H::BLOCK;
	const uint32_t nb = !g.hashed ? 0 : nfull + 1 +
	    (rem >= (uint32_t)(H::BLOCK - H::LENBYTES) ? 1 : 0);
	if (lane < G) {
		geo_m[lane] = g.off + 8 + dlen;
		geo_len[lane] = g.mlen;
		geo_nb[lane] = live ? nb : 0;
	}
	wave_lds_sync();
	uint32_t nbmax = 0;
	for (uint32_t d = 0; d < G; d++)
		nbmax = max(nbmax, geo_nb[d]);
	nbmax = __builtin_amdgcn_readfirstlane(nbmax);
	const uint32_t K = BW_ROWS / G;
	const uint32_t (*lmid)[16] = g.alt ? mid + 2 : mid;
	typename H::State s;
	load_mid<H>(lmid, 0, s);
	for (uint32_t c0 = 0; c0 < nbmax; c0 += K) {
		/* row `lane`: block c0 + lane % K of datagram lane / K */
		const uint32_t d = lane / K, k = c0 + lane % K;
		if (d < G && k < geo_nb[d]) {
			const uint32_t ml = geo_len[d];
			uint32_t w[NW32];
			bw_block<H>(base + geo_m[d], k, ml / H::BLOCK, ml % H::BLOCK,
			    geo_nb[d], ((uint64_t)ml + H::BLOCK) << 3, w);
			sched_row<H>(w, rows + lane * ROW);
		}
		wave_lds_sync();
		const uint32_t cnt = min(K, nbmax - c0);
		for (uint32_t b = 0; b < cnt; b++)
			if (c0 + b < nb)
				rounds_row<H>(s, rows + (dl * K + b) * ROW);
		wave_lds_sync();
	}
	/* outer: one block = inner digest || 0x80 || 0... || bit count */
	if (g.hashed) {
		uint32_t w[NW32];
#pragma unroll
		for (int j = 0; j < NW32; j++)
			w[j] = 0;
		const int dw = digest_words<H>(s, IS384, w);
#pragma unroll
		for (int j = 12; j < 16; j++)		/* SHA-384 keeps 12 words */
			if (j >= dw)
				w[j] = 0;
		w[dw] = 0x80000000u;
		const uint64_t obits = (uint64_t)(H::BLOCK + 4 * dw) << 3;
		w[NW32 - 2] = (uint32_t)(obits >> 32);
		w[NW32 - 1] = (uint32_t)obits;
		load_mid<H>(lmid, 1, s);
		H::compress(s, w);
	}
	materialize<H>(s);
	uint32_t o[16];
	H::out_words(s, o, IS384);
	__syncthreads();		/* wave 1's IVs are in LDS */
	if (!mine)
		return;
	const uint8_t *field = base + g.off + 8;
	if (MODE == HMAC_BURST_RX) {
		uint32_t code = g.st;
		if (g.ok) {		/* net2_buffer_cmp, packet.n2t:253-257 */
			uint32_t diff = 0;
			if (g.hashed) {
#pragma unroll
				for (uint32_t j = 0; j < dlen; j++)
					diff |= field[j] ^
					    ((o[j >> 2] >> (8 * (j & 3))) & 0xffu);
			}
			code = !g.hashed || diff != 0 ? PKT_BAD : PKT_OK;
		}
		if (rx.seq != nullptr) {
			rx.seq[i] = g.seq;
			rx.flags[i] = g.fl;
		}
		if (code == PKT_OK && ivlen > 0 && iv != nullptr &&
		    (g.fl & PKT_PH_ENCRYPTED)) {
			const uint8_t *src = reinterpret_cast<const uint8_t *>(ivw[lane]);
			uint8_t *dst = iv + i * ivlen;
			for (uint32_t b = 0; b < ivlen; b++)
				dst[b] = src[b];
		}
		result[i] = (uint8_t)code;
		return;
	}
	/* TX */
	if (rx.rec != nullptr) {
		uint8_t *r = rx.rec + i * (dlen + 16);
		if (g.hashed)
			store_digest<dlen>(r, o);
		*reinterpret_cast<uint4 *>(r + dlen) = make_uint4(
		    g.ok ? bswap32(g.seq) : 0u, g.ok ? bswap32(g.fl) : 0u,
		    (uint32_t)i, g.st);
		return;
	}
	if (g.hashed) {
		uint8_t *h = out + g.off;
#pragma unroll
		for (int b = 0; b < 4; b++) {
			h[b] = (uint8_t)(g.seq >> (24 - 8 * b));
			h[4 + b] = (uint8_t)(g.fl >> (24 - 8 * b));
		}
		store_digest<dlen>(h + 8, o);
	}
	result[i] = (uint8_t)g.st;
}

/* ---- length binning (counting sort by block count, longest first) ---- */

__device__ __forceinline__ uint32_t bin_of(uint32_t len, int blk_shift,
    int lenbytes, uint32_t nbins)
{
	/* total compressions the message needs, including padding */
	uint64_t nb = (((uint64_t)len + lenbytes + 1 + (1u << blk_shift) - 1) >>
	    blk_shift);
	uint32_t b = nb >= nbins ? nbins - 1 : (uint32_t)nb;
	return nbins - 1 - b;	/* descending block count */
}

/* Packets per thread in the binning: one workgroup bins a tile of
 * 256 x 16 = 4,096 packets (the whole 256-workgroup grid covers 1 M packets
 * with one tile each).  Every workgroup pays a fixed cost (clearing the
 * 2,048-bin LDS histogram, the histogram scan, its global atomics), so
 * fewer, larger tiles win down to 4,096 packets; 2,048 and 8,192 measured
 * slower (profiles/round1/binning_time_ab.txt, three-launch binning;
 * profiles/round4/bin_probe_items32_tiles8192.txt, this kernel). */
constexpr int kBinItems = 16;
#define NET2_BIN_TILE (256 * kBinItems)
/* A thread's kBinItems lengths, all loads issued before any is used. */
__device__ __forceinline__ void load_lens(const uint32_t *__restrict__ lens,
    uint64_t n, uint64_t i0, uint32_t (&len)[kBinItems])
{
#pragma unroll
	for (int k = 0; k < kBinItems; k++) {
		const uint64_t i = i0 + (uint64_t)k * 256;
		len[k] = i < n ? lens[i] : 0u;
	}
}

/*
 * Binning in one launch (round 4; until round 3 a memset, a count and a
 * scatter launch): the count, the global prefix and the scatter, no memset.
 * A persistent grid of G workgroups -- at most 256, and no more than the
 * device holds at once (the host caps G at the co-resident capacity of this
 * kernel, net2_bin_order) -- each looping over its 4,096-packet tiles:
 *   1. LDS histogram of its tiles, each packet's rank in its bin kept in
 *      registers (the LDS atomic's return value), then one device-scope
 *      fetch-add per touched bin into the global histogram, whose old value
 *      is where the workgroup's packets start inside that bin;
 *   2. a grid barrier in two levels: 16 group counters (workgroup
 *      blockIdx & 15, one XCD each), the last of each group arrives at a top
 *      counter, the last of those flips `state` to GO and bumps the epoch;
 *      everyone polls `state`;
 *   3. every workgroup scans the global histogram (8 KiB) for the bin
 *      bases and writes perm[base + start + rank] -- no claim pass, no
 *      second read of the lengths (a workgroup with several tiles ranks
 *      them again from the same starts).
 * The workspace cleans up after itself: the histogram and the barrier words
 * come in two parities (the epoch selects); each launch zeroes the parity
 * the next launch uses, so nothing waits for the last workgroup to leave.
 *
 * Never a hang, never a wrong order, and every fallback counted in the
 * header (net2_sha2_workspace_stats):
 *   - a barrier that does not complete within the timeout (the grid not
 *     co-resident, e.g. beside long kernels on other streams) is decided
 *     ABORT by one compare-and-swap on `state`, which every workgroup then
 *     follows: all write the identity order (perm[i] = i, hashing in
 *     submission order: correct, only slower), the header is marked for
 *     re-initialisation and NET2_BIN_W_ABORTS counts it;
 *   - a header is valid when its tag holds the magic and the id of a launch
 *     other than this one; otherwise (fresh memory, after an ABORT or a
 *     mismatch -- which leave a re-init mark, so the counters survive -- or
 *     prepared by workgroup 0 of this very launch -- a workgroup dispatched
 *     after workgroup 0 re-tagged it must not join a barrier the early ones
 *     skipped) every workgroup takes the identity order while workgroup 0
 *     initialises the header and both parities, so the next launch bins
 *     (NET2_BIN_W_UNPREP counts it);
 *   - after the barrier every workgroup checks that the global histogram
 *     adds up to n (64-bit sum): anything else -- stale counts, or barrier
 *     words someone else overwrote (a caller reusing the workspace for other
 *     data) -- marks the launch bad (NET2_BIN_W_BAD = its id,
 *     NET2_BIN_W_MISMATCH counts it) and clears the magic.  Workgroups that
 *     read the histogram at different times may then have written a mix of
 *     orders, so the hash kernel of this launch, given the same id, hashes
 *     in submission order instead (bin_perm);
 *   - the hash kernels clamp perm entries to [0, n) (a corrupt workspace
 *     can cost the binning, never an out-of-bounds access).
 * The workspace must not be used by two launches at once (as before).
 *
 * Memory ordering.  What crosses the barrier is the histogram, written and
 * read only by device-scope atomics, each workgroup's adds returned before
 * it arrives; the plain stores (perm, the next parity's zeroes) are read
 * only by later launches.  So the barrier needs no cache maintenance: its
 * atomics are relaxed.  On gfx950 an agent-scope release writes back the
 * XCD's L2 and an acquire invalidates it; with acq_rel arrivals and an
 * acquire fence the launch measured ~15 % longer, with an acquiring load
 * per poll ~3x (profiles/round4/bin_probe_*.txt).
 */
#define BIN_ORD __ATOMIC_RELAXED
constexpr int kBinSpinSleep = 2;
#define NET2_BIN_GROUPS 16
/*
 * Barrier words, per parity, in the workspace after the two histograms
 * (each word on its own 128-byte line): group counters at 32 g, the top counter
 * at 512, the state at 544.  Words 2,048-4,095 of the area hold the probe
 * stamps (NET2_BIN_PROBE=1, tools/bin_probe.py: thread 0 of every
 * workgroup stamps the 100 MHz clock at seven points; a measurement build,
 * never the shipped one).
 */
#define BIN_CTL_PAR 1024
#define BIN_CTL_TOP 512
#define BIN_CTL_STATE 544
#ifndef NET2_BIN_PROBE
#define NET2_BIN_PROBE 0
#endif
#define BIN_STAMP(p) do { if (NET2_BIN_PROBE && threadIdx.x == 0) \
	ctl0[2048 + blockIdx.x * 8 + (p)] = (uint32_t)wall_clock64(); } while (0)
#define NET2_BIN_MAGIC32 0x4e324253u	/* "N2BS" */
/* the tag after an ABORT or a mismatch: re-initialise, counters kept */
#define NET2_BIN_REINIT32 0x4e325249u	/* "N2RI" */
#define NET2_BIN_GRID 256
/* 50 ms of the 100 MHz s_memrealtime clock */
#define NET2_BIN_TIMEOUT 5000000ull
/* the first bin of packets that need at most two compressions */
#define NET2_BIN_SHORT (NET2_SHA2_NBINS - 3)

static_assert(NET2_BIN_CTL + 2048 + NET2_BIN_GRID * 8 <= NET2_BIN_WS_WORDS,
    "probe words");
static_assert(NET2_BIN_HDR + 2 * NET2_SHA2_NBINS <= NET2_BIN_CTL,
    "histograms");
static_assert(NET2_BIN_W_BINNED < NET2_BIN_HDR, "header words");
static_assert(BIN_CTL_STATE < BIN_CTL_PAR && 32 * NET2_BIN_GROUPS <= BIN_CTL_TOP,
    "barrier words");
static_assert(NET2_BIN_SHORT / (NET2_SHA2_NBINS / 256) == 255,
    "the short tail's first bin is the last thread's");
enum { BIN_UNDECIDED = 0, BIN_GO = 1, BIN_ABORT = 2 };

__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void add_agent(uint32_t *p, uint32_t v)
{
	(void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED,
	    __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t *bin_tag(uint32_t *ws)
{
	return reinterpret_cast<uint64_t *>(ws + NET2_BIN_W_TAG);
}

/* perm[i] = i for this workgroup's tiles */
__device__ __forceinline__ void bin_identity(uint32_t *perm, uint64_t n,
    uint64_t ntiles)
{
	for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x)
		for (int k = 0; k < kBinItems; k++) {
			const uint64_t i = t * NET2_BIN_TILE + (uint64_t)k * 256 +
			    threadIdx.x;
			if (i < n)
				perm[i] = (uint32_t)i;
		}
}

__global__ __launch_bounds__(256) void bin_onepass_kernel(
    const uint32_t *__restrict__ lens, uint64_t n, int blk_shift,
    int lenbytes, uint32_t *__restrict__ ws, uint64_t timeout,
    uint32_t launch)
{
	__shared__ uint32_t cnt[NET2_SHA2_NBINS];
	__shared__ uint32_t start[NET2_SHA2_NBINS];
	__shared__ uint32_t wsum[4];
	__shared__ uint64_t wtot[4];
	__shared__ uint32_t bc[2];
	uint32_t *hist0 = ws + NET2_BIN_HDR;		/* [2][NBINS] */
	uint32_t *ctl0 = ws + NET2_BIN_CTL;		/* [2][1024] */
	uint32_t *perm = ws + NET2_BIN_WS_WORDS;
	const uint32_t G = gridDim.x;
	const uint64_t ntiles = (n + NET2_BIN_TILE - 1) / NET2_BIN_TILE;
	constexpr uint32_t HW = NET2_SHA2_NBINS;

	/* the first tile's lengths in flight while the header is read */
	uint32_t len[kBinItems];
	load_lens(lens, n, (uint64_t)blockIdx.x * NET2_BIN_TILE + threadIdx.x,
	    len);
	if (threadIdx.x == 0) {
		const uint64_t tag = __hip_atomic_load(bin_tag(ws),
		    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		bc[0] = (uint32_t)(tag >> 32) == NET2_BIN_MAGIC32 &&
		    (uint32_t)tag != launch;
		bc[1] = ld_agent(&ws[NET2_BIN_W_EPOCH]);
	}
	for (uint32_t b = threadIdx.x; b < NET2_SHA2_NBINS; b += blockDim.x)
		cnt[b] = 0;
	__syncthreads();
	if (!bc[0]) {
		/* not initialised: submission order now, initialise for next */
		bin_identity(perm, n, ntiles);
		if (blockIdx.x == 0) {
			for (uint32_t w = threadIdx.x; w < 2 * HW; w += blockDim.x)
				hist0[w] = 0;
			for (uint32_t w = threadIdx.x; w < 2 * BIN_CTL_PAR;
			    w += blockDim.x)
				ctl0[w] = 0;
			if (threadIdx.x == 0) {
				/* fresh memory (no re-init mark): its counters
				 * are garbage, start them here */
				const uint64_t tag = __hip_atomic_load(bin_tag(ws),
				    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				if ((uint32_t)(tag >> 32) != NET2_BIN_REINIT32)
					for (int w = NET2_BIN_W_EPOCH + 1;
					    w <= NET2_BIN_W_BINNED; w++)
						ws[w] = 0;
				ws[NET2_BIN_W_EPOCH] = 0;
				add_agent(&ws[NET2_BIN_W_UNPREP], 1u);
			}
			__threadfence();
			__syncthreads();
			if (threadIdx.x == 0)
				__hip_atomic_store(bin_tag(ws),
				    (uint64_t)NET2_BIN_MAGIC32 << 32 | launch,
				    __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
		}
		return;
	}
	BIN_STAMP(0);
	const uint32_t par = bc[1] & 1;
	uint32_t *hist = hist0 + par * HW;
	uint32_t *ctl = ctl0 + par * BIN_CTL_PAR;
	/* the next launch's parity, zeroed: its histogram across the grid, its
	 * barrier words by workgroup 0 */
	for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < HW;
	    w += G * blockDim.x)
		hist0[(par ^ 1) * HW + w] = 0;
	if (blockIdx.x == 0 && threadIdx.x <= NET2_BIN_GROUPS + 1) {
		const uint32_t w = threadIdx.x < NET2_BIN_GROUPS ? 32 * threadIdx.x :
		    threadIdx.x == NET2_BIN_GROUPS ? BIN_CTL_TOP : BIN_CTL_STATE;
		ctl0[(par ^ 1) * BIN_CTL_PAR + w] = 0;
	}

	/* 1: this workgroup's histogram; the ranks of its first tile's packets
	 * kept in registers */
	uint32_t bin0[kBinItems], rank0[kBinItems];
	for (uint64_t t = blockIdx.x; t < ntiles; t += G) {
		const uint64_t i0 = t * NET2_BIN_TILE + threadIdx.x;
		if (t != blockIdx.x)
			load_lens(lens, n, i0, len);
#pragma unroll
		for (int k = 0; k < kBinItems; k++) {
			const uint32_t bn = bin_of(len[k], blk_shift, lenbytes,
			    NET2_SHA2_NBINS);
			const uint32_t r = i0 + (uint64_t)k * 256 < n ?
			    atomicAdd(&cnt[bn], 1u) : 0u;
			if (t == blockIdx.x) {
				bin0[k] = bn;
				rank0[k] = r;
			}
		}
	}
	__syncthreads();
	BIN_STAMP(1);
	/* into the global histogram: the add's old value is where this
	 * workgroup's packets start inside the bin */
	for (uint32_t b = threadIdx.x; b < NET2_SHA2_NBINS; b += blockDim.x)
		start[b] = cnt[b] != 0 ? __hip_atomic_fetch_add(&hist[b], cnt[b],
		    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
	__syncthreads();
	BIN_STAMP(2);

	/* 2: grid barrier in two levels, decided GO or ABORT exactly once */
	if (threadIdx.x == 0) {
		const uint32_t ng = G < NET2_BIN_GROUPS ? G : NET2_BIN_GROUPS;
		const uint32_t g = blockIdx.x % NET2_BIN_GROUPS;
		const uint32_t gsize = (G - g + NET2_BIN_GROUPS - 1) /
		    NET2_BIN_GROUPS;
		if (__hip_atomic_fetch_add(&ctl[32 * g], 1u, BIN_ORD,
		    __HIP_MEMORY_SCOPE_AGENT) == gsize - 1 &&
		    __hip_atomic_fetch_add(&ctl[BIN_CTL_TOP], 1u, BIN_ORD,
		    __HIP_MEMORY_SCOPE_AGENT) == ng - 1) {
			/* every workgroup has read the epoch by now */
			__hip_atomic_store(&ws[NET2_BIN_W_EPOCH], bc[1] + 1,
			    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			uint32_t exp = BIN_UNDECIDED;
			if (__hip_atomic_compare_exchange_strong(
			    &ctl[BIN_CTL_STATE], &exp, (uint32_t)BIN_GO, BIN_ORD,
			    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
				add_agent(&ws[NET2_BIN_W_BINNED], 1u);
		}
		BIN_STAMP(3);
		const uint64_t t0 = wall_clock64();
		uint32_t st;
		while ((st = ld_agent(&ctl[BIN_CTL_STATE])) == BIN_UNDECIDED) {
			if (wall_clock64() - t0 > timeout) {
				uint32_t exp = BIN_UNDECIDED;
				if (__hip_atomic_compare_exchange_strong(
				    &ctl[BIN_CTL_STATE], &exp,
				    (uint32_t)BIN_ABORT, BIN_ORD, __ATOMIC_RELAXED,
				    __HIP_MEMORY_SCOPE_AGENT))
					add_agent(&ws[NET2_BIN_W_ABORTS], 1u);
			}
			__builtin_amdgcn_s_sleep(kBinSpinSleep);
		}
		BIN_STAMP(4);
		bc[0] = st;
	}
	__syncthreads();
	bool binned = bc[0] == BIN_GO;
	if (binned) {
		/* 3: bin bases from the global histogram (8 bins per thread, a
		 * shuffle scan per wave, the four wave totals) added to the
		 * workgroup's starts, then its packets' places -- once the
		 * histogram is known to add up to n */
		constexpr int PER = NET2_SHA2_NBINS / 256;
		const int lane = (int)__lane_id(), wave = (int)(threadIdx.x / 64);
		/* (The histogram read with coalesced 8-byte loads staged through
		 * LDS, one request per line per workgroup instead of eight:
		 * 0.4 us slower to the bases -- the read is one round trip, not
		 * contention; profiles/round5/bin_probe_coalesced_read.txt.) */
		uint32_t v[PER], sum = 0;
		uint64_t sum64 = 0;
#pragma unroll
		for (int j = 0; j < PER; j++) {
			const uint32_t c = ld_agent(&hist[threadIdx.x * PER + j]);
			v[j] = sum;
			sum += c;
			sum64 += c;
		}
		uint32_t x = sum;
#pragma unroll
		for (int off = 1; off < 64; off <<= 1) {
			const uint32_t y = __shfl_up(x, off);
			if (lane >= off)
				x += y;
			sum64 += __shfl_xor(sum64, off);
		}
		if (lane == 63)
			wsum[wave] = x;
		if (lane == 0)
			wtot[wave] = sum64;
		__syncthreads();
		uint32_t base = x - sum;
		for (int w = 0; w < wave; w++)
			base += wsum[w];
		binned = wtot[0] + wtot[1] + wtot[2] + wtot[3] == n;
		if (binned) {
#pragma unroll
			for (int j = 0; j < PER; j++)
				start[threadIdx.x * PER + j] += base + v[j];
			/* where the packets of at most two compressions start */
			if (blockIdx.x == 0 && threadIdx.x == 255) {
				ws[NET2_BIN_W_TAIL] = base + v[NET2_BIN_SHORT % PER];
				ws[NET2_BIN_W_TAILID] = launch;
			}
		} else if (threadIdx.x == 0) {
			/* the histogram is not this launch's alone: the hash
			 * kernel of this launch ignores the order, and the next
			 * launch re-initialises */
			if (__hip_atomic_exchange(&ws[NET2_BIN_W_BAD], launch,
			    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != launch)
				add_agent(&ws[NET2_BIN_W_MISMATCH], 1u);
			__hip_atomic_store(bin_tag(ws),
			    (uint64_t)NET2_BIN_REINIT32 << 32, __ATOMIC_RELAXED,
			    __HIP_MEMORY_SCOPE_AGENT);
		}
		__syncthreads();
		BIN_STAMP(5);
	}
	if (binned) {
		if (ntiles <= G) {
			/* one tile: its packets' places from the kept ranks */
			const uint64_t i0 = (uint64_t)blockIdx.x * NET2_BIN_TILE +
			    threadIdx.x;
#pragma unroll
			for (int k = 0; k < kBinItems; k++) {
				const uint64_t i = i0 + (uint64_t)k * 256;
				const uint32_t pos = start[bin0[k]] + rank0[k];
				if (i < n && pos < n)
					perm[pos] = (uint32_t)i;
			}
		} else {
			/* several tiles: rank them again from the starts, one
			 * counter per bin */
			for (uint32_t b = threadIdx.x; b < NET2_SHA2_NBINS;
			    b += blockDim.x)
				cnt[b] = start[b];
			__syncthreads();
			for (uint64_t t = blockIdx.x; t < ntiles; t += G) {
				const uint64_t i0 = t * NET2_BIN_TILE + threadIdx.x;
				load_lens(lens, n, i0, len);
#pragma unroll
				for (int k = 0; k < kBinItems; k++) {
					const uint64_t i = i0 + (uint64_t)k * 256;
					if (i < n) {
						const uint32_t pos = atomicAdd(
						    &cnt[bin_of(len[k], blk_shift,
						    lenbytes, NET2_SHA2_NBINS)], 1u);
						if (pos < n)
							perm[pos] = (uint32_t)i;
					}
				}
			}
		}
		BIN_STAMP(6);
	} else {
		bin_identity(perm, n, ntiles);
		if (bc[0] != BIN_GO && threadIdx.x == 0) {
			/* ABORT: re-initialise at the next launch */
			__hip_atomic_store(bin_tag(ws),
			    (uint64_t)NET2_BIN_REINIT32 << 32, __ATOMIC_RELAXED,
			    __HIP_MEMORY_SCOPE_AGENT);
		}
	}
}

/* Prepares a binning workspace so its first launch bins, its counters
 * zeroed (one workgroup). */
__global__ __launch_bounds__(256) void bin_ws_init_kernel(uint32_t *ws)
{
	for (uint32_t w = threadIdx.x; w < NET2_BIN_WS_WORDS - 2;
	    w += blockDim.x)
		ws[2 + w] = 0;
	__threadfence();
	__syncthreads();
	if (threadIdx.x == 0)
		__hip_atomic_store(bin_tag(ws), (uint64_t)NET2_BIN_MAGIC32 << 32,
		    __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

/* ---- host-side constant pad schedule ---------------------------------- */

static inline uint32_t h_ror32(uint32_t x, int n)
{
	return (x >> n) | (x << (32 - n));
}
static inline uint64_t h_ror64(uint64_t x, int n)
{
	return (x >> n) | (x << (64 - n));
}

/* Pad block of a message whose length is a multiple of the block size. */
static void pad_kw256(uint64_t bits, PadKW<uint32_t> &p)
{
	uint32_t w[64] = { 0 };
	w[0] = 0x80000000u;
	w[14] = (uint32_t)(bits >> 32);
	w[15] = (uint32_t)bits;
	for (int t = 16; t < 64; t++) {
		uint32_t s0 = h_ror32(w[t - 15], 7) ^ h_ror32(w[t - 15], 18) ^
		    (w[t - 15] >> 3);
		uint32_t s1 = h_ror32(w[t - 2], 17) ^ h_ror32(w[t - 2], 19) ^
		    (w[t - 2] >> 10);
		w[t] = w[t - 16] + s0 + w[t - 7] + s1;
	}
	for (int t = 0; t < 64; t++)
		p.kw[t] = K256[t] + w[t];
}

static void pad_kw512(uint64_t bits, PadKW<uint64_t> &p)
{
	uint64_t w[80] = { 0 };
	w[0] = 0x8000000000000000ull;
	w[15] = bits;	/* w[14] = high 64 bits of the 128-bit count = 0 */
	for (int t = 16; t < 80; t++) {
		uint64_t s0 = h_ror64(w[t - 15], 1) ^ h_ror64(w[t - 15], 8) ^
		    (w[t - 15] >> 7);
		uint64_t s1 = h_ror64(w[t - 2], 19) ^ h_ror64(w[t - 2], 61) ^
		    (w[t - 2] >> 6);
		w[t] = w[t - 16] + s0 + w[t - 7] + s1;
	}
	for (int t = 0; t < 80; t++)
		p.kw[t] = K512[t] + w[t];
}

/*
 * The HMAC key blocks, once per launch on the host (RFC 2104 / FIPS 198-1:
 * the ipad and opad chaining values after one compression of K' ^ ipad /
 * K' ^ opad from the IV), in the word layout hmac_kernel's LDS copy takes.
 * One SHA-256 / SHA-512 compression each (FIPS 180-4 6.2.2 / 6.4.2, the
 * reference's SHA256Transform / SHA512Transform, src/sha2.c:374-445,
 * :663-734): product code of the launcher, not the test oracle.
 */
static void h_compress256(uint32_t st[8], const uint32_t m[16])
{
	uint32_t w[64], v[8];
	for (int t = 0; t < 16; t++)
		w[t] = m[t];
	for (int t = 16; t < 64; t++)
		w[t] = w[t - 16] + (h_ror32(w[t - 15], 7) ^ h_ror32(w[t - 15], 18) ^
		    (w[t - 15] >> 3)) + w[t - 7] + (h_ror32(w[t - 2], 17) ^
		    h_ror32(w[t - 2], 19) ^ (w[t - 2] >> 10));
	for (int i = 0; i < 8; i++)
		v[i] = st[i];
	for (int t = 0; t < 64; t++) {
		const uint32_t t1 = v[7] + (h_ror32(v[4], 6) ^ h_ror32(v[4], 11) ^
		    h_ror32(v[4], 25)) + ((v[4] & v[5]) ^ (~v[4] & v[6])) +
		    K256[t] + w[t];
		const uint32_t t2 = (h_ror32(v[0], 2) ^ h_ror32(v[0], 13) ^
		    h_ror32(v[0], 22)) + ((v[0] & v[1]) ^ (v[0] & v[2]) ^
		    (v[1] & v[2]));
		for (int i = 7; i > 0; i--)
			v[i] = v[i - 1];
		v[4] += t1;
		v[0] = t1 + t2;
	}
	for (int i = 0; i < 8; i++)
		st[i] += v[i];
}

static void h_compress512(uint64_t st[8], const uint64_t m[16])
{
	uint64_t w[80], v[8];
	for (int t = 0; t < 16; t++)
		w[t] = m[t];
	for (int t = 16; t < 80; t++)
		w[t] = w[t - 16] + (h_ror64(w[t - 15], 1) ^ h_ror64(w[t - 15], 8) ^
		    (w[t - 15] >> 7)) + w[t - 7] + (h_ror64(w[t - 2], 19) ^
		    h_ror64(w[t - 2], 61) ^ (w[t - 2] >> 6));
	for (int i = 0; i < 8; i++)
		v[i] = st[i];
	for (int t = 0; t < 80; t++) {
		const uint64_t t1 = v[7] + (h_ror64(v[4], 14) ^ h_ror64(v[4], 18) ^
		    h_ror64(v[4], 41)) + ((v[4] & v[5]) ^ (~v[4] & v[6])) +
		    K512[t] + w[t];
		const uint64_t t2 = (h_ror64(v[0], 28) ^ h_ror64(v[0], 34) ^
		    h_ror64(v[0], 39)) + ((v[0] & v[1]) ^ (v[0] & v[2]) ^
		    (v[1] & v[2]));
		for (int i = 7; i > 0; i--)
			v[i] = v[i - 1];
		v[4] += t1;
		v[0] = t1 + t2;
	}
	for (int i = 0; i < 8; i++)
		st[i] += v[i];
}

/*
 * ipad / opad midstates of key block kb (K' zero-padded to the block, at
 * most 128 bytes) into hm->w[slot], hm->w[slot + 1].  halg: the SHA row
 * (1 SHA-256, 2 SHA-384, 3 SHA-512).
 */
static void hmac_midstates(int halg, const uint8_t kb[128], HMid *hm,
    int slot)
{
	for (int pass = 0; pass < 2; pass++) {
		const uint8_t x = pass ? 0x5c : 0x36;
		uint32_t *o = hm->w[slot + pass];
		if (halg == 1) {
			uint32_t st[8], m[16];
			for (int i = 0; i < 8; i++)
				st[i] = IV256[i];
			for (int i = 0; i < 16; i++)
				m[i] = (uint32_t)(kb[4 * i] ^ x) << 24 |
				    (uint32_t)(kb[4 * i + 1] ^ x) << 16 |
				    (uint32_t)(kb[4 * i + 2] ^ x) << 8 |
				    (uint32_t)(kb[4 * i + 3] ^ x);
			h_compress256(st, m);
			for (int i = 0; i < 16; i++)
				o[i] = i < 8 ? st[i] : 0u;
		} else {
			uint64_t st[8], m[16];
			for (int i = 0; i < 8; i++)
				st[i] = halg == 2 ? IV384[i] : IV512[i];
			for (int i = 0; i < 16; i++) {
				uint64_t v = 0;
				for (int b = 0; b < 8; b++)
					v = v << 8 | (uint8_t)(kb[8 * i + b] ^ x);
				m[i] = v;
			}
			h_compress512(st, m);
			for (int i = 0; i < 8; i++) {
				o[2 * i] = (uint32_t)(st[i] >> 32);
				o[2 * i + 1] = (uint32_t)st[i];
			}
		}
	}
}

} /* namespace dev */
} /* namespace net2 */

#ifndef NET2_SHA2_NO_LAUNCHERS
/* ---- launch wrappers (C++ linkage, used by the C-ABI shim) ------------ */

using namespace net2::dev;

static inline unsigned grid_for(uint64_t n)
{
	return (unsigned)((n + 255) / 256);
}

hipError_t net2_launch_fixed(int alg, const uint8_t *base, uint64_t stride,
    uint32_t len, uint64_t n, uint8_t *out, hipStream_t s)
{
	const bool a16 = ((reinterpret_cast<uintptr_t>(base) | stride) & 15) == 0;
	const unsigned grid = grid_for(n);
	if (n == 0)
		return hipSuccess;
	if (alg == NET2_ALG_SHA256) {
		PadKW<uint32_t> pad;
		const bool padc = len % 64 == 0;
		if (padc)
			pad_kw256((uint64_t)len << 3, pad);
		if (a16 && padc)
			fixed_kernel<Sha256, AMODE_A16, true><<<grid, 256, 0, s>>>(
			    base, stride, len, n, out, 32, 0, pad);
		else if (a16)
			fixed_kernel<Sha256, AMODE_A16, false><<<grid, 256, 0, s>>>(
			    base, stride, len, n, out, 32, 0, pad);
		else
			fixed_kernel<Sha256, AMODE_A1, false><<<grid, 256, 0, s>>>(
			    base, stride, len, n, out, 32, 0, pad);
	} else {
		const int is384 = alg == NET2_ALG_SHA384;
		const uint32_t dlen = is384 ? 48 : 64;
		PadKW<uint64_t> pad;
		const bool padc = len % 128 == 0;
		if (padc)
			pad_kw512((uint64_t)len << 3, pad);
		if (a16 && padc)
			fixed_kernel<Sha512, AMODE_A16, true><<<grid, 256, 0, s>>>(
			    base, stride, len, n, out, dlen, is384, pad);
		else if (a16)
			fixed_kernel<Sha512, AMODE_A16, false><<<grid, 256, 0, s>>>(
			    base, stride, len, n, out, dlen, is384, pad);
		else
			fixed_kernel<Sha512, AMODE_A1, false><<<grid, 256, 0, s>>>(
			    base, stride, len, n, out, dlen, is384, pad);
	}
	return hipGetLastError();
}

hipError_t net2_bin_ws_init(uint32_t *ws, hipStream_t s)
{
	bin_ws_init_kernel<<<1, 256, 0, s>>>(ws);
	return hipGetLastError();
}

/*
 * Binning limits: the grid cap (0: the device's co-resident capacity) and
 * the barrier timeout in 100 MHz ticks, set by net2_sha2_bin_limits
 * (diagnostics and tests; read once per launch from two atomics, no
 * environment lookups on the launch path).
 */
static std::atomic<uint32_t> g_bin_grid_cap{0};
static std::atomic<uint64_t> g_bin_timeout{NET2_BIN_TIMEOUT};

void net2_bin_set_limits(uint32_t grid_cap, int64_t timeout_us)
{
	g_bin_grid_cap.store(grid_cap, std::memory_order_relaxed);
	g_bin_timeout.store(timeout_us < 0 ? NET2_BIN_TIMEOUT :
	    (uint64_t)timeout_us * 100, std::memory_order_relaxed);
}

/*
 * The persistent grid's size: at most 256 workgroups and no more than the
 * device can hold at once (workgroups per CU x CUs), cached per device --
 * on a partitioned device (a CPX partition has 32 CUs) 256 workgroups need
 * not all be resident, and the barrier would wait out its timeout on
 * every launch.
 */
static uint32_t bin_resident_grid()
{
	static std::atomic<uint32_t> cache[64];
	int dev = 0;
	if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
		(void)hipGetLastError();
		return NET2_BIN_GRID;
	}
	uint32_t g = cache[dev].load(std::memory_order_relaxed);
	if (g != 0)
		return g;
	int per_cu = 0, cus = 0;
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu,
	    bin_onepass_kernel, 256, 0) != hipSuccess ||
	    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount,
	    dev) != hipSuccess || per_cu <= 0 || cus <= 0) {
		(void)hipGetLastError();
		g = 1;		/* one workgroup is always resident */
	} else {
		g = (uint32_t)std::min<int64_t>(NET2_BIN_GRID,
		    (int64_t)per_cu * cus);
	}
	cache[dev].store(g, std::memory_order_relaxed);
	return g;
}

/* A launch id for the binning and the hash kernel that reads its order:
 * never 0 (the id of net2_bin_ws_init). */
static uint32_t next_bin_launch()
{
	static std::atomic<uint32_t> seq{0};
	uint32_t id;
	do
		id = seq.fetch_add(1, std::memory_order_relaxed) + 1;
	while (id == 0);
	return id;
}

/* Length-binned visiting order of a variable-length batch into ws. */
hipError_t net2_bin_order(int alg, const uint32_t *lens, uint64_t n,
    uint32_t *ws, hipStream_t s, uint32_t *launch)
{
	const bool s256 = alg == NET2_ALG_SHA256;
	const int blk_shift = s256 ? 6 : 7;
	const int lenbytes = s256 ? 8 : 16;
	const uint64_t tiles = (n + NET2_BIN_TILE - 1) / NET2_BIN_TILE;
	uint32_t cap = bin_resident_grid();
	const uint32_t forced = g_bin_grid_cap.load(std::memory_order_relaxed);
	if (forced != 0 && forced < cap)
		cap = forced;
	const unsigned g = (unsigned)(tiles < cap ? tiles : cap);
	*launch = next_bin_launch();
	bin_onepass_kernel<<<g, 256, 0, s>>>(lens, n, blk_shift, lenbytes, ws,
	    g_bin_timeout.load(std::memory_order_relaxed), *launch);
	return hipGetLastError();
}

hipError_t net2_launch_var(int alg, const uint8_t *base,
    const uint64_t *offsets, const uint32_t *lens, uint64_t n, uint8_t *out,
    uint32_t *ws, hipStream_t s)
{
	if (n == 0)
		return hipSuccess;
	const bool s256 = alg == NET2_ALG_SHA256;
	const int is384 = alg == NET2_ALG_SHA384;
	const uint32_t dlen = s256 ? 32 : is384 ? 48 : 64;
	uint32_t launch = 0;

	if (ws != nullptr) {
		hipError_t e = net2_bin_order(alg, lens, n, ws, s, &launch);
		if (e != hipSuccess)
			return e;
	}
	if (s256)
		var_kernel<Sha256V><<<grid_for(n), 256, 0, s>>>(base, offsets,
		    lens, ws, launch, n, out, dlen, 0);
	else
		var_kernel<Sha512V><<<grid_for(n), 256, 0, s>>>(base, offsets,
		    lens, ws, launch, n, out, dlen, is384);
	return hipGetLastError();
}
/* Every mode takes H's pair loop.  (Until round 5 the SHA-256 VERIFY and
 * BURST_RX kernels dropped it: 1.5 % faster in round 1, when the key pass
 * held their VGPRs at 110.  With the midstates from the host they measured
 * +4.3 to +5.3 % (verify) and +2.9 to +3.3 % (burst RX) with it,
 * profiles/round5/ab_pairall_box*.txt.) */

template <class H, bool IS384>
static void launch_hmac_var_mode(int mode, unsigned grid, hipStream_t s,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lens,
    const uint32_t *ws, uint32_t launch, uint64_t n, uint8_t *out,
    const HMid &hm, const PadKW<typename H::word> &pad, const BurstArgs &rx)
{
	if (mode == HMAC_SIGN)
		hmac_kernel<H, false, HMAC_SIGN, IS384><<<grid, 256, 0, s>>>(base,
		    offsets, lens, ws, launch, 0, 0, n, out, hm, pad, rx);
	else if (mode == HMAC_VERIFY)
		hmac_kernel<H, false, HMAC_VERIFY, IS384>
		    <<<grid, 256, 0, s>>>(base, offsets, lens, ws, launch, 0, 0, n,
		    out, hm, pad, rx);
	else if (mode == HMAC_BURST_RX)
		hmac_kernel<H, false, HMAC_BURST_RX, IS384>
		    <<<grid, 256, 0, s>>>(base, offsets, lens, ws, launch, 0, 0, n,
		    out, hm, pad, rx);
	else if (mode == HMAC_BURST_TX)
		hmac_kernel<H, false, HMAC_BURST_TX, IS384><<<grid, 256, 0, s>>>(
		    base, offsets, lens, ws, launch, 0, 0, n, out, hm, pad, rx);
	else
		hmac_kernel<H, false, HMAC_DIGESTS, IS384><<<grid, 256, 0, s>>>(
		    base, offsets, lens, ws, launch, 0, 0, n, out, hm, pad, rx);
}

/* The fixed layout (offsets == NULL): digests only. */
template <class H, bool IS384>
static void launch_hmac_fixed(bool padconst, unsigned grid, hipStream_t s,
    const uint8_t *base, uint64_t stride, uint32_t fixed_len, uint64_t n,
    uint8_t *out, const HMid &hm, const PadKW<typename H::word> &pad,
    const BurstArgs &rx)
{
	if (padconst)
		hmac_kernel<H, true, HMAC_DIGESTS, IS384><<<grid, 256, 0, s>>>(
		    base, nullptr, nullptr, nullptr, 0, stride, fixed_len, n, out,
		    hm, pad, rx);
	else
		hmac_kernel<H, false, HMAC_DIGESTS, IS384><<<grid, 256, 0, s>>>(
		    base, nullptr, nullptr, nullptr, 0, stride, fixed_len, n, out,
		    hm, pad, rx);
}

hipError_t net2_launch_hmac(int alg, const uint8_t *key, size_t keylen,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lens,
    uint64_t stride, uint32_t fixed_len, uint64_t n, uint8_t *out,
    uint32_t *ws, hipStream_t s, int mode, const BurstArgs *burst_args)
{
	if (mode != HMAC_DIGESTS && offsets == nullptr)
		return hipErrorInvalidValue;	/* datagram modes: var layout */
	if ((mode == HMAC_BURST_RX || mode == HMAC_BURST_TX) !=
	    (burst_args != nullptr))
		return hipErrorInvalidValue;
	if (burst_args != nullptr && burst_args->rec != nullptr &&
	    mode != HMAC_BURST_TX)
		return hipErrorInvalidValue;
	const BurstArgs rx = burst_args ? *burst_args : BurstArgs{};
	if (n == 0)
		return hipSuccess;
	const int halg = alg - 3;	/* HMAC row -> SHA row */
	const bool s256 = halg == NET2_ALG_SHA256;
	const int blk = s256 ? 64 : 128;
	const bool is384 = halg == NET2_ALG_SHA384;
	uint8_t kb[128] = { 0 };
	if (keylen > (size_t)blk)
		return hipErrorInvalidValue;	/* registry keys are <= a block */
	for (size_t i = 0; i < keylen; i++)
		kb[i] = key[i];
	HMid hm = {};
	hmac_midstates(halg, kb, &hm, 0);
	if (mode == HMAC_BURST_RX && rx.alt) {
		uint8_t ab[128] = { 0 };
		for (int i = 0; i < 32; i++)	/* K' as big-endian words */
			for (int b = 0; b < 4; b++)
				ab[4 * i + b] = (uint8_t)(rx.altkey[i] >> (24 - 8 * b));
		hmac_midstates(halg, ab, &hm, 2);
	}
	uint32_t launch = 0;
	if (offsets != nullptr && ws != nullptr) {
		hipError_t e = net2_bin_order(halg, lens, n, ws, s, &launch);
		if (e != hipSuccess)
			return e;
	} else {
		ws = nullptr;
	}
	const unsigned grid = grid_for(n);
	const bool padconst = offsets == nullptr && fixed_len % blk == 0;
	const uint64_t ibits = ((uint64_t)fixed_len + blk) << 3;
	if (s256) {
		PadKW<uint32_t> pad = {};
		if (offsets != nullptr) {
			launch_hmac_var_mode<Sha256H, false>(mode, grid, s, base,
			    offsets, lens, ws, launch, n, out, hm, pad, rx);
		} else {
			if (padconst)
				pad_kw256(ibits, pad);
			launch_hmac_fixed<Sha256H, false>(padconst, grid, s, base,
			    stride, fixed_len, n, out, hm, pad, rx);
		}
	} else {
		PadKW<uint64_t> pad = {};
		if (offsets != nullptr) {
			if (is384)
				launch_hmac_var_mode<Sha512H, true>(mode, grid, s, base,
				    offsets, lens, ws, launch, n, out, hm, pad, rx);
			else
				launch_hmac_var_mode<Sha512H, false>(mode, grid, s,
				    base, offsets, lens, ws, launch, n, out, hm, pad,
				    rx);
		} else {
			if (padconst)
				pad_kw512(ibits, pad);
			if (is384)
				launch_hmac_fixed<Sha512HF, true>(padconst, grid, s,
				    base, stride, fixed_len, n, out, hm, pad, rx);
			else
				launch_hmac_fixed<Sha512HF, false>(padconst, grid, s,
				    base, stride, fixed_len, n, out, hm, pad, rx);
		}
	}
	return hipGetLastError();
}
template <class H, bool IS384>
static void launch_burst_wave(int mode, uint64_t n, uint32_t G, hipStream_t s,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lens,
    const HMid &hm, const BurstArgs &a, uint8_t *result, uint8_t *iv,
    uint32_t ivlen, uint8_t *out)
{
	const unsigned grid = (unsigned)((n + G - 1) / G);
	if (mode == HMAC_BURST_RX)
		burst_wave_kernel<H, HMAC_BURST_RX, IS384><<<grid, 128, 0, s>>>(
		    base, offsets, lens, n, G, hm, a, result, iv, ivlen, out);
	else
		burst_wave_kernel<H, HMAC_BURST_TX, IS384><<<grid, 128, 0, s>>>(
		    base, offsets, lens, n, G, hm, a, result, iv, ivlen, out);
}

/* SIMDs of the current device (0: unknown), cached per ordinal. */
static uint64_t device_simds()
{
	static std::atomic<int> cus[64];
	int dev = 0;
	if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
		(void)hipGetLastError();
		return 0;
	}
	int c = cus[dev].load(std::memory_order_relaxed);
	if (c == 0) {
		if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount,
		    dev) != hipSuccess || c <= 0) {
			(void)hipGetLastError();
			return 0;
		}
		cus[dev].store(c, std::memory_order_relaxed);
	}
	return (uint64_t)c * 4;
}

/* net2_sha2_burst_limits' setting (-1: none) */
static std::atomic<int64_t> g_burst_wave_max{-1};

void net2_set_burst_wave_max(int64_t v)
{
	g_burst_wave_max.store(v < 0 ? -1 : v, std::memory_order_relaxed);
}

uint64_t net2_burst_wave_max(void)
{
	const int64_t set = g_burst_wave_max.load(std::memory_order_relaxed);
	if (set >= 0)
		return (uint64_t)set;
	/* NET2_BURST_WAVE_MAX, read once (A/B runs, one process per setting) */
	static const int64_t env = [] {
		const char *e = getenv("NET2_BURST_WAVE_MAX");
		return e != nullptr && *e != '\0' ?
		    (int64_t)(strtoull(e, nullptr, 10) & INT64_MAX) : (int64_t)-1;
	}();
	if (env >= 0)
		return (uint64_t)env;
	/* BW_GMAX datagrams per SIMD: beyond that a pass of the wave form
	 * expands too few blocks per datagram to beat the lane form */
	return device_simds() * BW_GMAX;
}

hipError_t net2_launch_burst_wave(int alg, const uint8_t *key, size_t keylen,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lens,
    uint64_t n, const BurstArgs *args, uint8_t *result, uint8_t *iv,
    uint32_t ivlen, uint8_t *out, int mode, hipStream_t s)
{
	if ((mode != HMAC_BURST_RX && mode != HMAC_BURST_TX) || args == nullptr ||
	    offsets == nullptr || ivlen > 64 || n > 0xffffffffu)
		return hipErrorInvalidValue;
	if (mode == HMAC_BURST_RX && args->rec != nullptr)
		return hipErrorInvalidValue;
	if (n == 0)
		return hipSuccess;
	const int halg = alg - 3;	/* HMAC row -> SHA row */
	const int blk = halg == NET2_ALG_SHA256 ? 64 : 128;
	if (halg < NET2_ALG_SHA256 || halg > NET2_ALG_SHA512 ||
	    keylen > (size_t)blk)
		return hipErrorInvalidValue;
	uint8_t kb[128] = { 0 };
	for (size_t j = 0; j < keylen; j++)
		kb[j] = key[j];
	HMid hm = {};
	hmac_midstates(halg, kb, &hm, 0);
	if (mode == HMAC_BURST_RX && args->alt) {
		uint8_t ab[128] = { 0 };
		for (int j = 0; j < 32; j++)	/* K' as big-endian words */
			for (int b = 0; b < 4; b++)
				ab[4 * j + b] = (uint8_t)(args->altkey[j] >> (24 - 8 * b));
		hmac_midstates(halg, ab, &hm, 2);
	}
	/* datagrams per workgroup: about one workgroup per SIMD */
	const uint64_t simds = std::max<uint64_t>(device_simds(), 1);
	const uint32_t G = (uint32_t)std::min<uint64_t>(BW_GMAX,
	    std::max<uint64_t>(1, (n + simds - 1) / simds));
	if (halg == NET2_ALG_SHA256)
		launch_burst_wave<Sha256H, false>(mode, n, G, s, base, offsets,
		    lens, hm, *args, result, iv, ivlen, out);
	else if (halg == NET2_ALG_SHA384)
		launch_burst_wave<Sha512H, true>(mode, n, G, s, base, offsets,
		    lens, hm, *args, result, iv, ivlen, out);
	else
		launch_burst_wave<Sha512H, false>(mode, n, G, s, base, offsets,
		    lens, hm, *args, result, iv, ivlen, out);
	return hipGetLastError();
}

hipError_t net2_launch_jobs(const uint8_t *stage, const Net2Job *jobs,
    uint32_t n256, uint32_t n512, uint8_t *out, uint32_t *done, int wave,
    hipStream_t s, uint32_t chunk)
{
	if (chunk == 0 || chunk % 128 != 0)
		return hipErrorInvalidValue;
	if (wave) {
		/* one 64-lane workgroup (one wave) per job */
		if (n256 > 0)
			job_wave_kernel<Sha256><<<n256, 64, 0, s>>>(stage, jobs,
			    out, done);
		if (n512 > 0)
			job_wave_kernel<Sha512><<<n512, 64, 0, s>>>(stage,
			    jobs + n256, out + 64 * (size_t)n256, done);
		return hipGetLastError();
	}
	/* 64-lane workgroups: a few jobs spread over as many CUs as waves */
	if (n256 > 0)
		job_kernel<Sha256><<<(n256 + 63) / 64, 64, 0, s>>>(stage, jobs,
		    n256, out, done, chunk);
	if (n512 > 0)
		job_kernel<Sha512J><<<(n512 + 63) / 64, 64, 0, s>>>(stage,
		    jobs + n256, n512, out + 64 * (size_t)n256, done, chunk);
	return hipGetLastError();
}

hipError_t net2_launch_burst_prep(uint8_t *base, const uint64_t *offsets,
    const uint32_t *lens, uint64_t n, int encode, int hash_set, int enc_set,
    uint32_t hashlen, const uint32_t *seq_in, const uint32_t *flags_in,
    uint32_t *seq_out, uint32_t *flags_out, uint64_t *sub_off,
    uint32_t *sub_len, uint8_t *status, hipStream_t s)
{
	burst_prep_kernel<<<grid_for(n), 256, 0, s>>>(base, offsets, lens, n,
	    encode, hash_set, enc_set, hashlen, seq_in, flags_in, seq_out,
	    flags_out, sub_off, sub_len, status);
	return hipGetLastError();
}

hipError_t net2_launch_burst_final(uint64_t n, const uint8_t *status,
    const uint8_t *verdict, const uint32_t *seq, const uint32_t *flags,
    uint32_t ivlen, uint8_t *iv, uint8_t *result, hipStream_t s,
    uint32_t *seq_out, uint32_t *flags_out)
{
	if (ivlen > 64 || (seq_out == nullptr) != (flags_out == nullptr))
		return hipErrorInvalidValue;
	if (n == 0)
		return hipSuccess;
	burst_final_kernel<<<grid_for(n), 256, 0, s>>>(n, status, verdict, seq,
	    flags, ivlen, iv, result, seq_out, flags_out);
	return hipGetLastError();
}

hipError_t net2_launch_ph_iv(const uint32_t *seq, const uint32_t *flags,
    uint64_t n, uint32_t ivlen, uint8_t *out, hipStream_t s)
{
	if (n == 0 || ivlen == 0)
		return hipSuccess;
	if (ivlen > 64)
		return hipErrorInvalidValue;
	ph_iv_kernel<<<grid_for(n), 256, 0, s>>>(seq, flags, n, ivlen, out);
	return hipGetLastError();
}
#endif /* NET2_SHA2_NO_LAUNCHERS */
