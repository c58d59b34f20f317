/*
 * sha2_device.h -- gfx950 device building blocks for the batched SHA-2 path.
 *
 * Replaces the per-block transforms of the reference (src/sha2.c:374-445
 * SHA256Transform, :663-734 SHA512Transform) with register-resident,
 * fully unrolled compressions written for CDNA4's integer VALU:
 *   - 32-bit rotates are one v_alignbit_b32 each;
 *   - three-input xor, Ch and Maj are one v_bitop3_b32 each;
 *   - the T1 sum folds into v_add3_u32;
 *   - big-endian message words come from one v_perm_b32 byte swap.
 * No MFMA: this is rotate/add/xor work, not a contraction.
 */
#ifndef NET2_SHA2_DEVICE_H
#define NET2_SHA2_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace net2 {
namespace dev {

/* FIPS 180-4 4.2.2: SHA-256 round constants (src/sha2.c:178-195). */
constexpr uint32_t K256[64] = {
	0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu,
	0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u, 0xd807aa98u, 0x12835b01u,
	0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u,
	0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu,
	0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u,
	0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u,
	0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
	0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
	0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u,
	0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u, 0x1e376c08u,
	0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu,
	0x682e6ff3u, 0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u,
	0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u,
};

/* FIPS 180-4 4.2.3: SHA-384/512 round constants (src/sha2.c:211-252). */
constexpr uint64_t K512[80] = {
	0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full,
	0xe9b5dba58189dbbcull, 0x3956c25bf348b538ull, 0x59f111f1b605d019ull,
	0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull, 0xd807aa98a3030242ull,
	0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
	0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull,
	0xc19bf174cf692694ull, 0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull,
	0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull, 0x2de92c6f592b0275ull,
	0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
	0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full,
	0xbf597fc7beef0ee4ull, 0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull,
	0x06ca6351e003826full, 0x142929670a0e6e70ull, 0x27b70a8546d22ffcull,
	0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
	0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull,
	0x92722c851482353bull, 0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull,
	0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull, 0xd192e819d6ef5218ull,
	0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
	0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull,
	0x34b0bcb5e19b48a8ull, 0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull,
	0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull, 0x748f82ee5defb2fcull,
	0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
	0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull,
	0xc67178f2e372532bull, 0xca273eceea26619cull, 0xd186b8c721c0c207ull,
	0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull, 0x06f067aa72176fbaull,
	0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
	0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull,
	0x431d67c49c100d4cull, 0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull,
	0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull,
};

/* Initial hash values, FIPS 180-4 5.3.3/5.3.4/5.3.5 (src/sha2.c:198-276). */
constexpr uint32_t IV256[8] = {
	0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
	0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u,
};
constexpr uint64_t IV384[8] = {
	0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull,
	0x152fecd8f70e5939ull, 0x67332667ffc00b31ull, 0x8eb44a8768581511ull,
	0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull,
};
constexpr uint64_t IV512[8] = {
	0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
	0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
	0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull,
};

/* ---- 32-bit primitives ------------------------------------------------ */

__device__ __forceinline__ uint32_t ror(uint32_t x, uint32_t n)
{
	return __builtin_amdgcn_alignbit(x, x, n);
}

/* bitop3 truth tables: bit (a<<2 | b<<1 | c) of the immediate. */
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
	return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

/*
 * Ch and Maj are spelled as explicit bitop3s: written as C expressions the
 * compiler splits Ch into v_and + v_bitop3 + an add folded into the T1 sum,
 * one extra VALU op per round.  Operand convention (checked against hipcc's
 * own bitop3 selection): S0 = 0xF0, S1 = 0xCC, S2 = 0xAA.
 */
__device__ __forceinline__ uint32_t ch32(uint32_t e, uint32_t f, uint32_t g)
{
	return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);	/* e ? f : g */
}

__device__ __forceinline__ uint32_t maj32(uint32_t a, uint32_t b, uint32_t c)
{
	return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);	/* majority */
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x)
{
	return __builtin_bswap32(x);
}

__device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t c)
{
	return a + b + c;	/* v_add3_u32 */
}

__device__ __forceinline__ uint32_t bsig0_256(uint32_t a)
{
	return xor3(ror(a, 2), ror(a, 13), ror(a, 22));
}
__device__ __forceinline__ uint32_t bsig1_256(uint32_t e)
{
	return xor3(ror(e, 6), ror(e, 11), ror(e, 25));
}
__device__ __forceinline__ uint32_t ssig0_256(uint32_t x)
{
	return xor3(ror(x, 7), ror(x, 18), x >> 3);
}
__device__ __forceinline__ uint32_t ssig1_256(uint32_t x)
{
	return xor3(ror(x, 17), ror(x, 19), x >> 10);
}

/*
 * One SHA-256 round.  The eight working variables live in s[] and are
 * renamed by index instead of being moved: at round t, variable a sits in
 * slot (0 - t) & 7, b in (1 - t) & 7, ..., h in (7 - t) & 7.  The new e
 * overwrites d's slot and the new a overwrites h's slot.  kw = K[t] + W[t]
 * already summed where the caller can (constant pad block), else the
 * caller passes K and W separately.
 */
/*
 * Ordered asm rounds (ASM = true, every kernel): the body of a round (and of a schedule word) is one
 * inline-asm block with a fixed instruction order: the six rotates of e and
 * a are independent of each other and are issued back to back, Ch/Maj and
 * the Sigma xors fill in between, the adds come last.  Left to itself the
 * machine scheduler orders each Sigma as rotate, rotate, rotate, xor --
 * every xor right behind the rotates it consumes -- and the same
 * instructions run 5 % slower (tools/sha_variants.hip V0 vs V6/V7,
 * profiles/round1/sha256_round_variants.json: identical instruction
 * multiset, only the order differs).  h + K + W stays outside the block so
 * the compiler can take K (or the pad block's K + W) from an SGPR.
 */
constexpr bool kAsm256 = true;
/* a scheduling fence every 2 rounds (see Rounds256) */
constexpr int kFence256 = 2;

/* The round body as one asm block (see above). */
__device__ __forceinline__ void round256_asm(uint32_t a, uint32_t b,
    uint32_t c, uint32_t &d, uint32_t e, uint32_t f, uint32_t g,
    uint32_t &h, uint32_t x)
{
	uint32_t r1, r2, r3, r4, r5;
	asm("v_alignbit_b32 %[r1], %[e], %[e], 6\n\t"
	    "v_alignbit_b32 %[r2], %[e], %[e], 11\n\t"
	    "v_alignbit_b32 %[r3], %[e], %[e], 25\n\t"
	    "v_alignbit_b32 %[r4], %[a], %[a], 2\n\t"
	    "v_alignbit_b32 %[r5], %[a], %[a], 13\n\t"
	    "v_bitop3_b32 %[r1], %[r1], %[r2], %[r3] bitop3:0x96\n\t"
	    "v_alignbit_b32 %[r2], %[a], %[a], 22\n\t"
	    "v_bitop3_b32 %[r3], %[e], %[f], %[g] bitop3:0xca\n\t"
	    "v_bitop3_b32 %[r4], %[r4], %[r5], %[r2] bitop3:0x96\n\t"
	    "v_bitop3_b32 %[r5], %[a], %[b], %[c] bitop3:0xe8\n\t"
	    "v_add3_u32 %[r1], %[x], %[r1], %[r3]\n\t"
	    "v_add_u32 %[d], %[d], %[r1]\n\t"
	    "v_add3_u32 %[h], %[r1], %[r4], %[r5]"
	    : [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [r4] "=&v"(r4),
	      [r5] "=&v"(r5), [h] "=v"(h), [d] "+v"(d)
	    : [a] "v"(a), [b] "v"(b), [c] "v"(c), [e] "v"(e), [f] "v"(f),
	      [g] "v"(g), [x] "v"(x));
}

template <int T, bool ASM = kAsm256>
__device__ __forceinline__ void round256(uint32_t (&s)[8], uint32_t k,
    uint32_t w)
{
	uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
	uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
	uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
	if (ASM) {
		round256_asm(a, b, c, d, e, f, g, h, add3(h, k, w));
	} else {
		uint32_t t1 = add3(add3(h, k, w), bsig1_256(e), ch32(e, f, g));
		d += t1;
		h = add3(t1, bsig0_256(a), maj32(a, b, c));
	}
}

/* sigma1(y) + w7 + sigma0(x) + w16 as one asm block (see round256_asm). */
__device__ __forceinline__ void expand256_asm(uint32_t &w16, uint32_t w7,
    uint32_t x, uint32_t y)
{
	uint32_t r1, r2, r3, r4, r5, r6;
	asm("v_alignbit_b32 %[r1], %[y], %[y], 17\n\t"
	    "v_alignbit_b32 %[r2], %[y], %[y], 19\n\t"
	    "v_alignbit_b32 %[r3], %[x], %[x], 7\n\t"
	    "v_alignbit_b32 %[r4], %[x], %[x], 18\n\t"
	    "v_lshrrev_b32 %[r5], 10, %[y]\n\t"
	    "v_lshrrev_b32 %[r6], 3, %[x]\n\t"
	    "v_bitop3_b32 %[r1], %[r1], %[r2], %[r5] bitop3:0x96\n\t"
	    "v_bitop3_b32 %[r3], %[r3], %[r4], %[r6] bitop3:0x96\n\t"
	    "v_add3_u32 %[w16], %[w16], %[r1], %[w7]\n\t"
	    "v_add_u32 %[w16], %[w16], %[r3]"
	    : [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [r4] "=&v"(r4),
	      [r5] "=&v"(r5), [r6] "=&v"(r6), [w16] "+v"(w16)
	    : [x] "v"(x), [y] "v"(y), [w7] "v"(w7));
}

/* W[t & 15] for t >= 16, in place over the 16-word circular schedule. */
template <int T, bool ASM = kAsm256>
__device__ __forceinline__ uint32_t expand256(uint32_t (&w)[16])
{
	if (ASM)
		expand256_asm(w[T & 15], w[(T - 7) & 15], w[(T - 15) & 15],
		    w[(T - 2) & 15]);
	else
		w[T & 15] = add3(w[T & 15], ssig1_256(w[(T - 2) & 15]),
		    w[(T - 7) & 15] + ssig0_256(w[(T - 15) & 15]));
	return w[T & 15];
}

template <int T, bool ASM>
struct Rounds256 {
	__device__ __forceinline__ static void run(uint32_t (&s)[8],
	    uint32_t (&w)[16])
	{
		uint32_t wt = T < 16 ? w[T & 15] : expand256<T, ASM>(w);
		round256<T, ASM>(s, K256[T], wt);
		/* keep the schedule words from being computed far ahead of
		 * their rounds (register pressure: 8 waves/SIMD need <= 64) */
		if (ASM && kFence256 > 0 && T % kFence256 == kFence256 - 1)
			__builtin_amdgcn_sched_barrier(0);
		Rounds256<T + 1, ASM>::run(s, w);
	}
};
template <bool ASM>
struct Rounds256<64, ASM> {
	__device__ __forceinline__ static void run(uint32_t (&)[8],
	    uint32_t (&)[16]) {}
};

/* SHA256Transform (src/sha2.c:374-445) on registers: st += F(st, w). */
template <bool ASM = kAsm256>
__device__ __forceinline__ void compress256(uint32_t (&st)[8],
    uint32_t (&w)[16])
{
	uint32_t s[8];
#pragma unroll
	for (int i = 0; i < 8; i++)
		s[i] = st[i];
	Rounds256<0, ASM>::run(s, w);
	/* After 64 rounds the renaming has wrapped around (64 % 8 == 0). */
#pragma unroll
	for (int i = 0; i < 8; i++)
		st[i] += s[i];
}

/*
 * Compression of a block whose whole schedule is known up front (the
 * constant padding block of a length that is a multiple of 64): kw[t] =
 * K[t] + W[t] comes precomputed from the host, so no expansion runs.
 */
template <int T, bool ASM>
struct RoundsKW256 {
	__device__ __forceinline__ static void run(uint32_t (&s)[8],
	    const uint32_t *kw)
	{
		round256<T, ASM>(s, kw[T], 0u);
		if (ASM && kFence256 > 0 && T % kFence256 == kFence256 - 1)
			__builtin_amdgcn_sched_barrier(0);
		RoundsKW256<T + 1, ASM>::run(s, kw);
	}
};
template <bool ASM>
struct RoundsKW256<64, ASM> {
	__device__ __forceinline__ static void run(uint32_t (&)[8],
	    const uint32_t *) {}
};

template <bool ASM = kAsm256>
__device__ __forceinline__ void compress256_kw(uint32_t (&st)[8],
    const uint32_t *kw)
{
	uint32_t s[8];
#pragma unroll
	for (int i = 0; i < 8; i++)
		s[i] = st[i];
	RoundsKW256<0, ASM>::run(s, kw);
#pragma unroll
	for (int i = 0; i < 8; i++)
		st[i] += s[i];
}

/* ---- 64-bit primitives on 32-bit lanes ----------------------------------- */

/*
 * 64-bit words are register pairs.  Halves are moved in and out with
 * bit casts of a two-lane vector, never with (hi << 32) | lo: written as
 * shift/or, LLVM re-splits sums of such values into extra v_mov and 64-bit
 * adds (measured: +10% VALU per SHA-512 block).
 */
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t lo32(uint64_t x)
{
	return __builtin_bit_cast(u32x2, x).x;
}
__device__ __forceinline__ uint32_t hi32(uint64_t x)
{
	return __builtin_bit_cast(u32x2, x).y;
}
__device__ __forceinline__ uint64_t mk64(uint32_t lo, uint32_t hi)
{
	u32x2 v = { lo, hi };
	return __builtin_bit_cast(uint64_t, v);
}

/* 64-bit rotate right = two v_alignbit_b32 (halves swap when N >= 32). */
template <int N>
__device__ __forceinline__ uint64_t ror64(uint64_t x)
{
	uint32_t l = lo32(x), h = hi32(x);
	if (N < 32)
		return mk64(__builtin_amdgcn_alignbit(h, l, N),
		    __builtin_amdgcn_alignbit(l, h, N));
	return mk64(__builtin_amdgcn_alignbit(l, h, N - 32),
	    __builtin_amdgcn_alignbit(h, l, N - 32));
}

__device__ __forceinline__ uint64_t xor3_64(uint64_t a, uint64_t b,
    uint64_t c)
{
	return mk64(xor3(lo32(a), lo32(b), lo32(c)),
	    xor3(hi32(a), hi32(b), hi32(c)));
}

__device__ __forceinline__ uint64_t ch64(uint64_t e, uint64_t f, uint64_t g)
{
	return mk64(ch32(lo32(e), lo32(f), lo32(g)),
	    ch32(hi32(e), hi32(f), hi32(g)));
}

__device__ __forceinline__ uint64_t maj64(uint64_t a, uint64_t b, uint64_t c)
{
	return mk64(maj32(lo32(a), lo32(b), lo32(c)),
	    maj32(hi32(a), hi32(b), hi32(c)));
}

__device__ __forceinline__ uint64_t bswap64(uint64_t x)
{
	return mk64(bswap32(hi32(x)), bswap32(lo32(x)));
}

__device__ __forceinline__ uint64_t bsig0_512(uint64_t a)
{
	return xor3_64(ror64<28>(a), ror64<34>(a), ror64<39>(a));
}
__device__ __forceinline__ uint64_t bsig1_512(uint64_t e)
{
	return xor3_64(ror64<14>(e), ror64<18>(e), ror64<41>(e));
}
/*
 * 64-bit logical shift as one v_lshrrev_b64 (hipcc otherwise emits
 * v_alignbit_b32 + v_lshrrev_b32, two VALU ops for the same result).
 * Issue costs (tools/valu_probe): v_lshrrev_b64 4.2 SIMD cycles per wave
 * instruction against 4.3 + 2.6 for the pair; measured -2% on the SHA-512
 * fixed kernel (profiles/round1/sha512_u2_shr_ab.json).
 */
template <int N>
__device__ __forceinline__ uint64_t shr64(uint64_t x)
{
	uint64_t r;
	asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "i"(N), "v"(x));
	return r;
}

__device__ __forceinline__ uint64_t ssig0_512(uint64_t x)
{
	return xor3_64(ror64<1>(x), ror64<8>(x), shr64<7>(x));
}
__device__ __forceinline__ uint64_t ssig1_512(uint64_t x)
{
	return xor3_64(ror64<19>(x), ror64<61>(x), shr64<6>(x));
}

/*
 * The bitwise half of a SHA-512 round -- the 12 rotates of Sigma1(e) and
 * Sigma0(a) (two v_alignbit_b32 per 64-bit rotate) and the 8 v_bitop3_b32 of
 * the Sigma xors, Ch and Maj -- as one asm block with a fixed order (rotates
 * first), as round256_asm does for SHA-256; the 64-bit sums stay in C
 * (v_lshl_add_u64 needs register pairs, which inline asm cannot split into
 * halves).  Three other orders measured within 1 % on C4, c3_512 and
 * hmac512_mtu (profiles/round2/sha512_order_ab.txt) and were removed.
 */
__device__ __forceinline__ void bitwise512_asm(uint64_t a, uint64_t b,
    uint64_t c, uint64_t e, uint64_t f, uint64_t g, uint64_t &S1,
    uint64_t &CH, uint64_t &S0, uint64_t &MJ)
{
	uint32_t r1, r2, r3, r4, r5, r6;
	uint32_t s1l, s1h, chl, chh, s0l, s0h, mjl, mjh;
	/* rotr n < 32: lo = alignbit(hi, lo, n), hi = alignbit(lo, hi, n);
	 * rotr 32 + m: lo = alignbit(lo, hi, m), hi = alignbit(hi, lo, m) */
	asm("v_alignbit_b32 %[r1], %[eh], %[el], 14\n\t"
	    "v_alignbit_b32 %[r2], %[eh], %[el], 18\n\t"
	    "v_alignbit_b32 %[r3], %[el], %[eh], 9\n\t"
	    "v_alignbit_b32 %[r4], %[el], %[eh], 14\n\t"
	    "v_alignbit_b32 %[r5], %[el], %[eh], 18\n\t"
	    "v_alignbit_b32 %[r6], %[eh], %[el], 9\n\t"
	    "v_bitop3_b32 %[s1l], %[r1], %[r2], %[r3] bitop3:0x96\n\t"
	    "v_bitop3_b32 %[s1h], %[r4], %[r5], %[r6] bitop3:0x96\n\t"
	    "v_alignbit_b32 %[r1], %[ah], %[al], 28\n\t"
	    "v_alignbit_b32 %[r2], %[al], %[ah], 2\n\t"
	    "v_alignbit_b32 %[r3], %[al], %[ah], 7\n\t"
	    "v_alignbit_b32 %[r4], %[al], %[ah], 28\n\t"
	    "v_alignbit_b32 %[r5], %[ah], %[al], 2\n\t"
	    "v_alignbit_b32 %[r6], %[ah], %[al], 7\n\t"
	    "v_bitop3_b32 %[chl], %[el], %[fl], %[gl] bitop3:0xca\n\t"
	    "v_bitop3_b32 %[chh], %[eh], %[fh], %[gh] bitop3:0xca\n\t"
	    "v_bitop3_b32 %[s0l], %[r1], %[r2], %[r3] bitop3:0x96\n\t"
	    "v_bitop3_b32 %[s0h], %[r4], %[r5], %[r6] bitop3:0x96\n\t"
	    "v_bitop3_b32 %[mjl], %[al], %[bl], %[cl] bitop3:0xe8\n\t"
	    "v_bitop3_b32 %[mjh], %[ah], %[bh], %[ch] bitop3:0xe8"
	    : [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [r4] "=&v"(r4),
	      [r5] "=&v"(r5), [r6] "=&v"(r6),
	      [s1l] "=&v"(s1l), [s1h] "=&v"(s1h),
	      [chl] "=&v"(chl), [chh] "=&v"(chh), [s0l] "=&v"(s0l),
	      [s0h] "=&v"(s0h), [mjl] "=&v"(mjl), [mjh] "=&v"(mjh)
	    : [al] "v"(lo32(a)), [ah] "v"(hi32(a)), [bl] "v"(lo32(b)),
	      [bh] "v"(hi32(b)), [cl] "v"(lo32(c)), [ch] "v"(hi32(c)),
	      [el] "v"(lo32(e)), [eh] "v"(hi32(e)), [fl] "v"(lo32(f)),
	      [fh] "v"(hi32(f)), [gl] "v"(lo32(g)), [gh] "v"(hi32(g)));
	S1 = mk64(s1l, s1h);
	CH = mk64(chl, chh);
	S0 = mk64(s0l, s0h);
	MJ = mk64(mjl, mjh);
}

template <int T>
__device__ __forceinline__ void round512(uint64_t (&s)[8], uint64_t kw)
{
	uint64_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
	uint64_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
	uint64_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
	uint64_t S1, CH, S0, MJ;
	bitwise512_asm(a, b, c, e, f, g, S1, CH, S0, MJ);
	uint64_t t1 = h + kw + S1 + CH;
	d += t1;
	h = t1 + S0 + MJ;
}

/*
 * sigma0(x) and sigma1(y) of a SHA-512 schedule word with the rotates in one
 * ordered asm block (as bitwise512_asm); the 64-bit shifts (v_lshrrev_b64) are
 * passed in, their halves read directly.
 */
__device__ __forceinline__ void ssigmas512_asm(uint64_t x, uint64_t y,
    uint64_t xs, uint64_t ys, uint64_t &P0, uint64_t &P1)
{
	uint32_t r1, r2, r3, r4, p0l, p0h, p1l, p1h;
	asm("v_alignbit_b32 %[r1], %[yh], %[yl], 19\n\t"
	    "v_alignbit_b32 %[r2], %[yl], %[yh], 29\n\t"
	    "v_alignbit_b32 %[r3], %[yl], %[yh], 19\n\t"
	    "v_alignbit_b32 %[r4], %[yh], %[yl], 29\n\t"
	    "v_bitop3_b32 %[p1l], %[r1], %[r2], %[ysl] bitop3:0x96\n\t"
	    "v_bitop3_b32 %[p1h], %[r3], %[r4], %[ysh] bitop3:0x96\n\t"
	    "v_alignbit_b32 %[r1], %[xh], %[xl], 1\n\t"
	    "v_alignbit_b32 %[r2], %[xh], %[xl], 8\n\t"
	    "v_alignbit_b32 %[r3], %[xl], %[xh], 1\n\t"
	    "v_alignbit_b32 %[r4], %[xl], %[xh], 8\n\t"
	    "v_bitop3_b32 %[p0l], %[r1], %[r2], %[xsl] bitop3:0x96\n\t"
	    "v_bitop3_b32 %[p0h], %[r3], %[r4], %[xsh] bitop3:0x96"
	    : [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [r4] "=&v"(r4),
	      [p0l] "=&v"(p0l), [p0h] "=&v"(p0h), [p1l] "=&v"(p1l),
	      [p1h] "=&v"(p1h)
	    : [xl] "v"(lo32(x)), [xh] "v"(hi32(x)), [yl] "v"(lo32(y)),
	      [yh] "v"(hi32(y)), [xsl] "v"(lo32(xs)), [xsh] "v"(hi32(xs)),
	      [ysl] "v"(lo32(ys)), [ysh] "v"(hi32(ys)));
	P0 = mk64(p0l, p0h);
	P1 = mk64(p1l, p1h);
}

template <int T>
__device__ __forceinline__ uint64_t expand512(uint64_t (&w)[16])
{
	const uint64_t x = w[(T - 15) & 15], y = w[(T - 2) & 15];
	uint64_t P0, P1;
	ssigmas512_asm(x, y, shr64<7>(x), shr64<6>(y), P0, P1);
	w[T & 15] += P1 + w[(T - 7) & 15] + P0;
	return w[T & 15];
}

/*
 * W[t] + K[t] for SHA-512: a per-workgroup LDS copy of K (k512_lds, filled
 * by k512_lds_fill() at kernel entry), read with one broadcast ds_read_b64
 * per round, so the constant costs an LDS issue slot instead of VALU time or
 * SGPRs (left as plain C constants, hipcc parks all 80 in SGPR pairs and
 * spills ~100 SGPRs into VGPR lanes).  The reads are plain (non-volatile)
 * loads through a base address offset by an opaque per-compression zero (an
 * `s_mov_b32 0` the compiler cannot see through): loop-variant, so not
 * hoisted out of the block loop (which would pin 160 VGPRs), yet free to
 * move with the rounds that consume them (a volatile read cannot be sunk:
 * when a compression's result is used only under a lane condition, the
 * compiler sank the rounds into the branch and left all 80 reads above it,
 * live at once -- HMAC-SHA512 reached 400 VGPRs).
 */
typedef __attribute__((address_space(3))) uint64_t lds_k64;
__shared__ uint64_t k512_lds[160];	/* [0,80) K512, [80,160) pad K+W */

/*
 * Every thread of the workgroup must call one of these before any SHA-512
 * round.  The padded variant also copies the host-precomputed K[t] + W[t]
 * of the constant padding block (a kernel argument, 80 64-bit words) to
 * k512_lds[80 + t]: left in the kernel argument it would be hoisted into 160
 * SGPRs and spilled.  The argument is read with constant indices only (an
 * address-taken by-value argument is copied to scratch by hipcc).
 */
__device__ __forceinline__ void k512_lds_fill()
{
	for (unsigned i = threadIdx.x; i < 80; i += blockDim.x)
		k512_lds[i] = K512[i];
	__syncthreads();
}

template <class PAD>
__device__ __forceinline__ void k512_lds_fill_pad(const PAD &pad)
{
	for (unsigned i = threadIdx.x; i < 80; i += blockDim.x)
		k512_lds[i] = K512[i];
	if (threadIdx.x < 64) {
		/* lane l stores pad words l and l + 64 (constant-index reads,
		 * selected per lane) */
#pragma unroll
		for (int t = 0; t < 64; t++)
			if (threadIdx.x == (unsigned)t)
				k512_lds[80 + t] = pad.kw[t];
#pragma unroll
		for (int t = 64; t < 80; t++)
			if (threadIdx.x == (unsigned)(t - 64))
				k512_lds[80 + t] = pad.kw[t];
	}
	__syncthreads();
}

/* Base of the LDS constant table for one compression (the opaque zero). */
__device__ __forceinline__ const lds_k64 *k512_base()
{
	uint32_t z;
	asm volatile("s_mov_b32 %0, 0" : "=s"(z));
	return (const lds_k64 *)k512_lds + z;
}

template <int T>
__device__ __forceinline__ uint64_t k512_at(const lds_k64 *kb)
{
	return kb[T];
}

template <int T>
__device__ __forceinline__ uint64_t addk512(uint64_t w, const lds_k64 *kb)
{
	return w + k512_at<T>(kb);
}

template <int T>
struct Rounds512 {
	__device__ __forceinline__ static void run(uint64_t (&s)[8],
	    uint64_t (&w)[16], const lds_k64 *kb)
	{
		uint64_t wt = T < 16 ? w[T & 15] : expand512<T>(w);
		round512<T>(s, addk512<T>(wt, kb));
		Rounds512<T + 1>::run(s, w, kb);
	}
};
template <>
struct Rounds512<80> {
	__device__ __forceinline__ static void run(uint64_t (&)[8],
	    uint64_t (&)[16], const lds_k64 *) {}
};

/* SHA512Transform (src/sha2.c:663-734) on registers. */
__device__ __forceinline__ void compress512(uint64_t (&st)[8],
    uint64_t (&w)[16])
{
	uint64_t s[8];
#pragma unroll
	for (int i = 0; i < 8; i++)
		s[i] = st[i];
	Rounds512<0>::run(s, w, k512_base());
#pragma unroll
	for (int i = 0; i < 8; i++)
		st[i] += s[i];
}

template <int T>
struct RoundsKW512 {
	__device__ __forceinline__ static void run(uint64_t (&s)[8],
	    const uint64_t *kw, const lds_k64 *kb)
	{
		/* the pad block's K + W sit in k512_lds[80, 160) */
		round512<T>(s, k512_at<80 + T>(kb));
		(void)kw;
		RoundsKW512<T + 1>::run(s, kw, kb);
	}
};
template <>
struct RoundsKW512<80> {
	__device__ __forceinline__ static void run(uint64_t (&)[8],
	    const uint64_t *, const lds_k64 *) {}
};

__device__ __forceinline__ void compress512_kw(uint64_t (&st)[8],
    const uint64_t *kw)
{
	uint64_t s[8];
#pragma unroll
	for (int i = 0; i < 8; i++)
		s[i] = st[i];
	RoundsKW512<0>::run(s, kw, k512_base());
#pragma unroll
	for (int i = 0; i < 8; i++)
		st[i] += s[i];
}

} /* namespace dev */
} /* namespace net2 */

#endif /* NET2_SHA2_DEVICE_H */
