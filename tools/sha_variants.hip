// sha_variants.hip -- A/B of SHA-256 round formulations on gfx950.
// Compute-only: every lane runs NBLK compressions on register-resident
// message words (no memory traffic), full grid of 16384 waves (the config-2
// wave count), so the timing isolates VALU issue cost.  All variants must
// produce identical states; the harness checks that.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sha_variants.hip -o tools/sha_variants
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
#include <algorithm>

#define NBLK 17
#ifndef WPE
#define WPE 1
#endif

__device__ constexpr uint32_t K256[64] = {
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

// ---- primitive forms -------------------------------------------------------
__device__ __forceinline__ uint32_t rot_ab(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t x3_b3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ uint32_t ch_b3(uint32_t e, uint32_t f, uint32_t g) { return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA); }
__device__ __forceinline__ uint32_t mj_b3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8); }

__device__ __forceinline__ uint32_t a_add(uint32_t a, uint32_t b) { uint32_t r; asm("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
template <uint32_t K>
__device__ __forceinline__ uint32_t a_addk(uint32_t a) { uint32_t r; asm("v_add_u32 %0, %1, %2" : "=v"(r) : "i"(K), "v"(a)); return r; }
__device__ __forceinline__ uint32_t a_add3(uint32_t a, uint32_t b, uint32_t c) { uint32_t r; asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c)); return r; }
__device__ __forceinline__ uint32_t a_xor(uint32_t a, uint32_t b) { uint32_t r; asm("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ uint32_t a_and(uint32_t a, uint32_t b) { uint32_t r; asm("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
template <int N>
__device__ __forceinline__ uint32_t a_shr(uint32_t a) { uint32_t r; asm("v_lshrrev_b32 %0, %1, %2" : "=v"(r) : "i"(N), "v"(a)); return r; }
template <int N>
__device__ __forceinline__ uint32_t a_shl(uint32_t a) { uint32_t r; asm("v_lshlrev_b32 %0, %1, %2" : "=v"(r) : "i"(N), "v"(a)); return r; }
template <int N>
__device__ __forceinline__ uint32_t a_rot(uint32_t a) { uint32_t r; asm("v_alignbit_b32 %0, %1, %1, %2" : "=v"(r) : "v"(a), "i"(N)); return r; }

// ---- variants ----------------------------------------------------------------
// V0: compiler-chosen from builtins (the shipped kernel's formulation)
struct V0 {
	template <int T> __device__ static void rnd(uint32_t (&s)[8], uint32_t w) {
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		uint32_t t1 = (h + K256[T] + w) + x3_b3(rot_ab(e, 6), rot_ab(e, 11), rot_ab(e, 25)) + ch_b3(e, f, g);
		d += t1;
		h = t1 + x3_b3(rot_ab(a, 2), rot_ab(a, 13), rot_ab(a, 22)) + mj_b3(a, b, c);
	}
	template <int T> __device__ static uint32_t exp(uint32_t (&w)[16]) {
		uint32_t x = w[(T - 15) & 15], y = w[(T - 2) & 15];
		w[T & 15] += x3_b3(rot_ab(y, 17), rot_ab(y, 19), y >> 10) + w[(T - 7) & 15] + x3_b3(rot_ab(x, 7), rot_ab(x, 18), x >> 3);
		return w[T & 15];
	}
};

// V1: K as a VOP2 literal (W + K), all other adds VOP2 (no add3), xor pairs
struct V1 {
	template <int T> __device__ static void rnd(uint32_t (&s)[8], uint32_t w) {
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		uint32_t s1 = a_xor(a_xor(a_rot<6>(e), a_rot<11>(e)), a_rot<25>(e));
		uint32_t t1 = a_add(a_add(a_add(a_addk<K256[T]>(w), h), s1), ch_b3(e, f, g));
		d = a_add(d, t1);
		uint32_t s0 = a_xor(a_xor(a_rot<2>(a), a_rot<13>(a)), a_rot<22>(a));
		h = a_add(a_add(t1, s0), mj_b3(a, b, c));
	}
	template <int T> __device__ static uint32_t exp(uint32_t (&w)[16]) {
		uint32_t x = w[(T - 15) & 15], y = w[(T - 2) & 15];
		uint32_t s1 = a_xor(a_xor(a_rot<17>(y), a_rot<19>(y)), a_shr<10>(y));
		uint32_t s0 = a_xor(a_xor(a_rot<7>(x), a_rot<18>(x)), a_shr<3>(x));
		w[T & 15] = a_add(a_add(a_add(w[T & 15], s1), w[(T - 7) & 15]), s0);
		return w[T & 15];
	}
};

// V2: like V1 but xor3 via bitop3 and the 3-term adds via add3
struct V2 {
	template <int T> __device__ static void rnd(uint32_t (&s)[8], uint32_t w) {
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		uint32_t s1 = x3_b3(a_rot<6>(e), a_rot<11>(e), a_rot<25>(e));
		uint32_t t1 = a_add3(a_add(a_addk<K256[T]>(w), h), s1, ch_b3(e, f, g));
		d = a_add(d, t1);
		uint32_t s0 = x3_b3(a_rot<2>(a), a_rot<13>(a), a_rot<22>(a));
		h = a_add3(t1, s0, mj_b3(a, b, c));
	}
	template <int T> __device__ static uint32_t exp(uint32_t (&w)[16]) {
		uint32_t x = w[(T - 15) & 15], y = w[(T - 2) & 15];
		uint32_t s1 = x3_b3(a_rot<17>(y), a_rot<19>(y), a_shr<10>(y));
		uint32_t s0 = x3_b3(a_rot<7>(x), a_rot<18>(x), a_shr<3>(x));
		w[T & 15] = a_add3(a_add(w[T & 15], s1), w[(T - 7) & 15], s0);
		return w[T & 15];
	}
};

// V3: V1 with Ch/Maj from VOP2 logic (Ch = ((f^g)&e)^g; Maj = b ^ ((a^b)&(b^c)))
struct V3 {
	template <int T> __device__ static void rnd(uint32_t (&s)[8], uint32_t w) {
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		uint32_t s1 = a_xor(a_xor(a_rot<6>(e), a_rot<11>(e)), a_rot<25>(e));
		uint32_t ch = a_xor(a_and(a_xor(f, g), e), g);
		uint32_t t1 = a_add(a_add(a_add(a_addk<K256[T]>(w), h), s1), ch);
		d = a_add(d, t1);
		uint32_t s0 = a_xor(a_xor(a_rot<2>(a), a_rot<13>(a)), a_rot<22>(a));
		uint32_t mj = a_xor(a_and(a_xor(a, b), a_xor(b, c)), b);
		h = a_add(a_add(t1, s0), mj);
	}
	template <int T> __device__ static uint32_t exp(uint32_t (&w)[16]) { return V1::exp<T>(w); }
};

// V4: rotations from shifts: rotr(x,n) = (x >> n) ^ (x << (32-n)), all xor VOP2
struct V4 {
	template <int N> __device__ static uint32_t rot(uint32_t x) { return a_xor(a_shr<N>(x), a_shl<32 - N>(x)); }
	template <int T> __device__ static void rnd(uint32_t (&s)[8], uint32_t w) {
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		uint32_t s1 = a_xor(a_xor(rot<6>(e), rot<11>(e)), rot<25>(e));
		uint32_t t1 = a_add(a_add(a_add(a_addk<K256[T]>(w), h), s1), ch_b3(e, f, g));
		d = a_add(d, t1);
		uint32_t s0 = a_xor(a_xor(rot<2>(a), rot<13>(a)), rot<22>(a));
		h = a_add(a_add(t1, s0), mj_b3(a, b, c));
	}
	template <int T> __device__ static uint32_t exp(uint32_t (&w)[16]) { return V1::exp<T>(w); }
};

// V5: V2 but adds: (W+K) literal, then add3(h, wk, s1) and add(ch) -- mix bitop3/add
struct V5 {
	template <int T> __device__ static void rnd(uint32_t (&s)[8], uint32_t w) {
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		uint32_t s1 = x3_b3(a_rot<6>(e), a_rot<11>(e), a_rot<25>(e));
		uint32_t t1 = a_add(a_add(a_add(a_addk<K256[T]>(w), h), s1), ch_b3(e, f, g));
		d = a_add(d, t1);
		uint32_t s0 = x3_b3(a_rot<2>(a), a_rot<13>(a), a_rot<22>(a));
		h = a_add(a_add(t1, s0), mj_b3(a, b, c));
	}
	template <int T> __device__ static uint32_t exp(uint32_t (&w)[16]) {
		uint32_t x = w[(T - 15) & 15], y = w[(T - 2) & 15];
		uint32_t s1 = x3_b3(a_rot<17>(y), a_rot<19>(y), a_shr<10>(y));
		uint32_t s0 = x3_b3(a_rot<7>(x), a_rot<18>(x), a_shr<3>(x));
		w[T & 15] = a_add(a_add(a_add(w[T & 15], s1), w[(T - 7) & 15]), s0);
		return w[T & 15];
	}
};


// V6: each round / schedule word as one asm block, slow-class instructions
// (alignbit, add3) grouped apart from fast-class ones (bitop3, add, lshr):
// tests whether slow<->fast issue transitions cost cycles (valu_probe "mix").
struct V6 {
	template <int T> __device__ static void rnd(uint32_t (&s)[8], uint32_t w) {
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		uint32_t r1, r2, r3, r4, r5, r6, x, t1;
		asm("v_alignbit_b32 %[r1], %[e], %[e], 6\n\t"
		    "v_alignbit_b32 %[r2], %[e], %[e], 11\n\t"
		    "v_alignbit_b32 %[r3], %[e], %[e], 25\n\t"
		    "v_alignbit_b32 %[r4], %[a], %[a], 2\n\t"
		    "v_alignbit_b32 %[r5], %[a], %[a], 13\n\t"
		    "v_alignbit_b32 %[r6], %[a], %[a], 22\n\t"
		    "v_add3_u32 %[x], %[h], %[k], %[w]\n\t"
		    "v_bitop3_b32 %[r1], %[r1], %[r2], %[r3] bitop3:0x96\n\t"
		    "v_bitop3_b32 %[r2], %[e], %[f], %[g] bitop3:0xca\n\t"
		    "v_bitop3_b32 %[r4], %[r4], %[r5], %[r6] bitop3:0x96\n\t"
		    "v_bitop3_b32 %[r5], %[a], %[b], %[c] bitop3:0xe8\n\t"
		    "v_add3_u32 %[t1], %[x], %[r1], %[r2]\n\t"
		    "v_add3_u32 %[h], %[t1], %[r4], %[r5]\n\t"
		    "v_add_u32 %[d], %[d], %[t1]"
		    : [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [r4] "=&v"(r4),
		      [r5] "=&v"(r5), [r6] "=&v"(r6), [x] "=&v"(x), [t1] "=&v"(t1),
		      [h] "+v"(h), [d] "+v"(d)
		    : [a] "v"(a), [b] "v"(b), [c] "v"(c), [e] "v"(e), [f] "v"(f),
		      [g] "v"(g), [k] "s"(K256[T]), [w] "v"(w));
	}
	template <int T> __device__ static uint32_t exp(uint32_t (&w)[16]) {
		uint32_t x = w[(T - 15) & 15], y = w[(T - 2) & 15];
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
		      [r5] "=&v"(r5), [r6] "=&v"(r6), [w16] "+v"(w[T & 15])
		    : [x] "v"(x), [y] "v"(y), [w7] "v"(w[(T - 7) & 15]));
		return w[T & 15];
	}
};

// V7: V6 order but interleaved slow/fast as much as dependencies allow
struct V7 {
	template <int T> __device__ static void rnd(uint32_t (&s)[8], uint32_t w) {
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		uint32_t r1, r2, r3, r4, r5, r6, x, t1;
		asm("v_alignbit_b32 %[r1], %[e], %[e], 6\n\t"
		    "v_bitop3_b32 %[r6], %[e], %[f], %[g] bitop3:0xca\n\t"
		    "v_alignbit_b32 %[r2], %[e], %[e], 11\n\t"
		    "v_bitop3_b32 %[r5], %[a], %[b], %[c] bitop3:0xe8\n\t"
		    "v_alignbit_b32 %[r3], %[e], %[e], 25\n\t"
		    "v_alignbit_b32 %[r4], %[a], %[a], 2\n\t"
		    "v_bitop3_b32 %[r1], %[r1], %[r2], %[r3] bitop3:0x96\n\t"
		    "v_alignbit_b32 %[r2], %[a], %[a], 13\n\t"
		    "v_alignbit_b32 %[r3], %[a], %[a], 22\n\t"
		    "v_add3_u32 %[x], %[h], %[k], %[w]\n\t"
		    "v_bitop3_b32 %[r4], %[r4], %[r2], %[r3] bitop3:0x96\n\t"
		    "v_add3_u32 %[t1], %[x], %[r1], %[r6]\n\t"
		    "v_add_u32 %[d], %[d], %[t1]\n\t"
		    "v_add3_u32 %[h], %[t1], %[r4], %[r5]"
		    : [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3), [r4] "=&v"(r4),
		      [r5] "=&v"(r5), [r6] "=&v"(r6), [x] "=&v"(x), [t1] "=&v"(t1),
		      [h] "+v"(h), [d] "+v"(d)
		    : [a] "v"(a), [b] "v"(b), [c] "v"(c), [e] "v"(e), [f] "v"(f),
		      [g] "v"(g), [k] "s"(K256[T]), [w] "v"(w));
	}
	template <int T> __device__ static uint32_t exp(uint32_t (&w)[16]) { return V6::exp<T>(w); }
};

// V8: builtins, V6's order written in the source; V9: V8 + a scheduling
// barrier after every round (no inline asm, so no hazard s_nops)
template <bool FENCE>
struct V8T {
	template <int T> __device__ static void rnd(uint32_t (&s)[8], uint32_t w) {
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		uint32_t r1 = rot_ab(e, 6), r2 = rot_ab(e, 11), r3 = rot_ab(e, 25);
		uint32_t r4 = rot_ab(a, 2), r5 = rot_ab(a, 13), r6 = rot_ab(a, 22);
		uint32_t x = h + K256[T] + w;
		uint32_t s1 = x3_b3(r1, r2, r3), ch = ch_b3(e, f, g);
		uint32_t s0 = x3_b3(r4, r5, r6), mj = mj_b3(a, b, c);
		uint32_t t1 = x + s1 + ch;
		h = t1 + s0 + mj;
		d += t1;
		if (FENCE)
			__builtin_amdgcn_sched_barrier(0);
	}
	template <int T> __device__ static uint32_t exp(uint32_t (&w)[16]) {
		uint32_t x = w[(T - 15) & 15], y = w[(T - 2) & 15];
		uint32_t r1 = rot_ab(y, 17), r2 = rot_ab(y, 19), r3 = rot_ab(x, 7), r4 = rot_ab(x, 18);
		uint32_t s1 = x3_b3(r1, r2, y >> 10), s0 = x3_b3(r3, r4, x >> 3);
		w[T & 15] = w[T & 15] + s1 + w[(T - 7) & 15] + s0;
		return w[T & 15];
	}
};
typedef V8T<false> V8;
typedef V8T<true> V9;

template <class V, int T>
struct R {
	__device__ __forceinline__ static void run(uint32_t (&s)[8], uint32_t (&w)[16]) {
		uint32_t wt = T < 16 ? w[T & 15] : V::template exp<T>(w);
		V::template rnd<T>(s, wt);
		R<V, T + 1>::run(s, w);
	}
};
template <class V>
struct R<V, 64> { __device__ __forceinline__ static void run(uint32_t (&)[8], uint32_t (&)[16]) {} };

template <class V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void kern(uint32_t *out, uint32_t seed)
{
	uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
	    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
	const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
	uint32_t x = gid * 0x9E3779B9u + seed;
	for (int blk = 0; blk < NBLK; blk++) {
		uint32_t w[16];
#pragma unroll
		for (int i = 0; i < 16; i++) {
			x = x * 1664525u + 1013904223u;
			w[i] = x;
		}
		uint32_t s[8];
#pragma unroll
		for (int i = 0; i < 8; i++) s[i] = st[i];
		R<V, 0>::run(s, w);
#pragma unroll
		for (int i = 0; i < 8; i++) st[i] += s[i];
	}
#pragma unroll
	for (int i = 0; i < 8; i++) out[gid * 8 + i] = st[i];
}

template <class V>
static float timeit(uint32_t *out, int blocks)
{
	hipEvent_t a, b;
	(void)hipEventCreate(&a); (void)hipEventCreate(&b);
	kern<V><<<blocks, 256>>>(out, 7);
	(void)hipDeviceSynchronize();
	(void)hipEventRecord(a);
	for (int i = 0; i < 5; i++) kern<V><<<blocks, 256>>>(out, 7);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms; (void)hipEventElapsedTime(&ms, a, b);
	return ms / 5;
}

int main()
{
	const int blocks = 4096;  // 16384 waves
	const size_t n = (size_t)blocks * 256 * 8;
	uint32_t *out;
	(void)hipMalloc(&out, n * 4 * 10);
	std::vector<uint32_t> ref(n), got(n);
	const char *names[] = {"V0 builtins (shipped)", "V1 VOP2 adds+xor, K literal", "V2 bitop3+add3, K literal",
	    "V3 VOP2 logic Ch/Maj", "V4 shift rotations", "V5 bitop3 + VOP2 adds",
	    "V6 asm rounds, slow/fast grouped", "V7 asm rounds, slow/fast interleaved",
	    "V8 builtins in V6 order", "V9 V8 + sched_barrier per round"};
	float best[10] = {1e9, 1e9, 1e9, 1e9, 1e9, 1e9, 1e9, 1e9, 1e9, 1e9};
	for (int round = 0; round < 3; round++) {
		best[0] = std::min(best[0], timeit<V0>(out + 0 * n, blocks));
		best[1] = std::min(best[1], timeit<V1>(out + 1 * n, blocks));
		best[2] = std::min(best[2], timeit<V2>(out + 2 * n, blocks));
		best[3] = std::min(best[3], timeit<V3>(out + 3 * n, blocks));
		best[4] = std::min(best[4], timeit<V4>(out + 4 * n, blocks));
		best[5] = std::min(best[5], timeit<V5>(out + 5 * n, blocks));
		best[6] = std::min(best[6], timeit<V6>(out + 6 * n, blocks));
		best[7] = std::min(best[7], timeit<V7>(out + 7 * n, blocks));
		best[8] = std::min(best[8], timeit<V8>(out + 8 * n, blocks));
		best[9] = std::min(best[9], timeit<V9>(out + 9 * n, blocks));
	}
	(void)hipMemcpy(ref.data(), out, n * 4, hipMemcpyDeviceToHost);
	printf("{\"blocks_per_lane\": %d, \"waves\": %d, \"variants\": [\n", NBLK, blocks * 4);
	for (int v = 0; v < 10; v++) {
		(void)hipMemcpy(got.data(), out + v * n, n * 4, hipMemcpyDeviceToHost);
		bool same = got == ref;
		double per_block_ns = best[v] * 1e6 / ((double)blocks * 256 * NBLK);
		printf("  {\"variant\": \"%s\", \"ms\": %.4f, \"same_as_V0\": %s, \"ps_per_lane_block\": %.3f}%s\n",
		    names[v], best[v], same ? "true" : "false", per_block_ns * 1e3, v == 9 ? "" : ",");
	}
	printf("]}\n");
	return 0;
}
