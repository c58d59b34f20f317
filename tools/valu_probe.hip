// valu_probe.hip -- issue cost of the integer VALU instructions the SHA-2
// rounds can be built from, measured on a full MI355X grid.
// Each probe runs CHAINS independent dependency chains per lane so latency
// is hidden; WPS = waves per SIMD (blocks of 256 threads per CU x 4 / 4).
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o tools/valu_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <vector>

#define CHAINS 8
#define ITERS 2048

// Operand forms as they appear in the SHA kernels.
#define BODY(K)                                                                   \
	if (K == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[c]) : "v"(b));     \
	if (K == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[c]) : "v"(b));     \
	if (K == 2) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(r[c]));           \
	if (K == 3) asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(r[c]));           \
	if (K == 4) asm volatile("v_or_b32 %0, %0, %1" : "+v"(r[c]) : "v"(b));      \
	if (K == 5) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[c]) : "v"(b), "v"(d)); \
	if (K == 6) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[c]));      \
	if (K == 7) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(r[c]) : "v"(b)); \
	if (K == 8) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(b), "v"(d)); \
	if (K == 9) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(b), "s"(s)); \
	if (K == 10) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(b), "v"(d)); \
	if (K == 11) asm volatile("v_perm_b32 %0, 0, %0, %1" : "+v"(r[c]) : "s"(s)); \
	if (K == 12) asm volatile("v_add_u32 %0, 0x428a2f98, %0" : "+v"(r[c]));     \
	if (K == 13) asm volatile("v_add_u32 %0, %1, %0" : "+v"(r[c]) : "s"(s));    \
	if (K == 14) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(b), "v"(d)); \
	if (K == 15) asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(r[c]) : "v"(b)); \
	if (K == 16) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(b), "v"(d)); \
	if (K == 17) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(r[c]) : "v"(b)); \
	if (K == 18) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(r[c]) : "v"(b)); \
	if (K == 19) asm volatile("v_mov_b32 %0, %1" : "=v"(r[c]) : "v"(r[(c + 1) % CHAINS])); \
	if (K == 20) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(r[c]) : "v"(b), "v"(d)); \
	if (K == 21) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(b), "v"(d)); \
	if (K == 22) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(b), "v"(d)); \
	if (K == 23) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(r[c]) : "v"(b)); \
	if (K == 24) asm volatile("v_lshrrev_b32_e64 %0, 7, %0" : "+v"(r[c]));       \
	if (K == 25) { if (c & 1) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[c])); \
	               else asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[c]) : "v"(b)); } \
	if (K == 26) { if (c & 1) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[c])); \
	               else asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(b), "v"(d)); } \
	if (K == 27) { if (c % 3 == 0) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[c])); \
	               else asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[c]) : "v"(b)); } \
	if (K == 28) { if (c & 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[c]) : "v"(b), "v"(d)); \
	               else asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[c]) : "v"(b)); } \
	if (K == 29) { if (c & 1) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[c])); \
	               else asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(r[c])); } \
	if (K == 30) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[c]) : "v"(bq)); \
	if (K == 31) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %2\n\tv_addc_co_u32_e32 %1, vcc, %1, %3, vcc" \
	                          : "+v"(r[c]), "+v"(r2[c]) : "v"(b), "v"(d) : "vcc"); \
	if (K == 32) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(q[c])); \
	if (K == 33) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[c]) : "s"(sq)); \
	if (K == 34) asm volatile("v_alignbit_b32 %0, %0, %0, %1" : "+v"(r[c]) : "s"(s)); \
	if (K == 35) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(q[c]) : "v"(bq)); \
	if (K == 36) asm volatile("v_add_f32_e32 %0, %0, %1" : "+v"(r[c]) : "v"(b)); \
	if (K == 37) asm volatile("v_and_b32_e32 %0, %0, %1" : "+v"(r[c]) : "v"(b)); \
	if (K == 38) asm volatile("v_not_b32_e32 %0, %0" : "+v"(r[c])); \
	if (K == 39) asm volatile("v_sub_u32_e32 %0, %0, %1" : "+v"(r[c]) : "v"(b)); \
	if (K == 40) { if (c & 1) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[c])); \
	               else asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[c]) : "v"(b), "v"(d)); } \
	if (K == 41) { if (c & 1) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(b), "v"(d)); \
	               else asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[c]) : "v"(b)); } \
	if (K == 42) asm volatile("v_lshlrev_b32_e32 %0, %1, %0" : "+v"(r[c]) : "v"(b)); \
	if (K == 43) asm volatile("v_mul_u32_u24_e32 %0, 0x80, %0" : "+v"(r[c])); \
	if (K == 44) { if (c < 4) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[c])); \
	               else asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[c]) : "v"(b)); } \
	if (K == 45) { if (c < 4) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(b), "v"(d)); \
	               else asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[c]) : "v"(b)); } \
	if (K == 46) asm volatile("v_bitop3_b32 %0, %0, %0, %0 bitop3:0x96" : "+v"(r[c])); \
	if (K == 47) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(r[c]) : "v"(r[(c + 1) % CHAINS]), "v"(r[(c + 2) % CHAINS])); \
	if (K == 48) asm volatile("v_add3_u32 %0, %1, %2, %0" : "+v"(r[c]) : "v"(r[(c + 1) % CHAINS]), "v"(r[(c + 2) % CHAINS])); \
	if (K == 49) asm volatile("v_alignbit_b32 %0, %1, %1, 7" : "=v"(r[c]) : "v"(r[(c + 3) % CHAINS]));

static const char *kNames[] = {
	"v_add_u32 (VOP2, v,v)", "v_xor_b32 (VOP2)", "v_lshrrev_b32 (VOP2, imm)",
	"v_lshlrev_b32 (VOP2, imm)", "v_or_b32 (VOP2)",
	"v_bitop3_b32 xor3 (3 v)", "v_alignbit_b32 x,x,imm (rotate)",
	"v_alignbit_b32 x,y,imm", "v_alignbit_b32 x,y,z", "v_add3_u32 v,v,s",
	"v_add3_u32 v,v,v", "v_perm_b32 0,v,s (bswap)", "v_add_u32 literal",
	"v_add_u32 s", "v_bfi_b32", "v_lshl_or_b32 v,imm,v", "v_xad_u32",
	"v_add_u32_e64 (VOP3 enc)", "v_alignbyte_b32 imm", "v_mov_b32",
	"v_bitop3_b32 ch (0xca)", "v_and_or_b32", "v_or3_b32", "v_xor_b32_e64",
	"v_lshrrev_b32_e64",
	"mix alignbit|xor 1:1", "mix alignbit|add3 1:1", "mix alignbit|xor 1:2",
	"mix bitop3|add 1:1", "mix alignbit|lshr 1:1",
	"v_lshl_add_u64 v,0,v (64-bit add)", "v_add_co_u32 + v_addc_co_u32 (VOP2 pair, per instr)",
	"v_lshrrev_b64 imm", "v_lshl_add_u64 v,0,s", "v_alignbit_b32 x,x,s",
	"v_pk_add_f32", "v_add_f32", "v_and_b32", "v_not_b32", "v_sub_u32",
	"mix alignbit|bitop3 1:1", "mix add3|add 1:1", "v_lshlrev_b32 v,v (VOP2 var shift)",
	"v_mul_u32_u24 literal",
	"grouped alignbit x4 | xor x4", "grouped add3 x4 | add x4",
	"v_bitop3_b32 x,x,x", "v_bitop3_b32 chain-mixed srcs", "v_add3_u32 chain-mixed srcs",
	"v_alignbit_b32 from other chain",
};
#define NK 50

template <int K>
__global__ __launch_bounds__(256) void probe(uint32_t *out, uint32_t seed)
{
	uint64_t t0 = __builtin_amdgcn_s_memtime();
	uint32_t r[CHAINS], r2[CHAINS];
	uint64_t q[CHAINS];
	uint64_t bq = ((uint64_t)seed << 32) ^ threadIdx.x;
	uint64_t sq = __builtin_amdgcn_readfirstlane(seed * 5 + 1);
	uint32_t b = seed ^ threadIdx.x, d = seed * 7 + threadIdx.x;
	uint32_t s = __builtin_amdgcn_readfirstlane(seed * 3 + 1);
#pragma unroll
	for (int c = 0; c < CHAINS; c++)
		r[c] = threadIdx.x * (c + 1), r2[c] = r[c] ^ seed, q[c] = ((uint64_t)r[c] << 32) | r2[c];
	for (int it = 0; it < ITERS; it++) {
#pragma unroll
		for (int c = 0; c < CHAINS; c++) {
			BODY(K)
		}
	}
	uint32_t x = 0;
#pragma unroll
	for (int c = 0; c < CHAINS; c++)
		x ^= r[c] ^ r2[c] ^ (uint32_t)q[c] ^ (uint32_t)(q[c] >> 32);
	if (x == 0x12345678u)
		out[0] = x;
	uint64_t t1 = __builtin_amdgcn_s_memtime();
	if ((threadIdx.x & 63) == 0)
		out[16 + blockIdx.x * 4 + threadIdx.x / 64] = (uint32_t)(t1 - t0);
}

template <class F>
static float time_kernel(F launch)
{
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	launch();
	(void)hipDeviceSynchronize();
	(void)hipEventRecord(a);
	for (int i = 0; i < 5; i++)
		launch();
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	return ms / 5;
}

template <int K>
static void run(uint32_t *out, int cus, int wps, bool last)
{
	const int blocks = cus * wps;  // wps blocks of 4 waves per CU -> wps waves / SIMD
	float ms = time_kernel([&] { probe<K><<<blocks, 256>>>(out, 1); });
	double instr = (double)blocks * 4 * ITERS * CHAINS * (K == 31 ? 2 : 1);  // wave instructions
	// cycles per wave-instruction per SIMD at the nominal 2.4 GHz
	double cyc = ms * 1e-3 * 2.4e9 * cus * 4 / instr;
	// clock-independent: median per-wave s_memtime span / (wps * instr per wave)
	static uint32_t h[16 + 256 * 8 * 4];
	(void)hipMemcpy(h, out, sizeof(uint32_t) * (16 + blocks * 4), hipMemcpyDeviceToHost);
	std::vector<uint32_t> v(h + 16, h + 16 + blocks * 4);
	std::sort(v.begin(), v.end());
	double span = v[v.size() / 2];
	double memcyc = span / (wps * (double)ITERS * CHAINS * (K == 31 ? 2 : 1));
	double clk = (double)v[v.size() - 1] / (ms * 1e-3) / 1e9;
	printf("  {\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, "
	    "\"simd_cycles_per_wave_instr_at_2.4GHz\": %.3f, \"memtime_cycles_per_wave_instr\": %.3f, \"memtime_GHz_est\": %.3f}%s\n",
	    kNames[K], wps, ms, cyc, memcyc, clk, last ? "" : ",");
}

template <int K>
static void run_all(uint32_t *out, int cus)
{
	run<K>(out, cus, 8, false);
	if constexpr (K + 1 < NK)
		run_all<K + 1>(out, cus);
}

int main()
{
	uint32_t *out;
	(void)hipMalloc(&out, sizeof(uint32_t) * (16 + 256 * 8 * 4));
	hipDeviceProp_t p;
	(void)hipGetDeviceProperties(&p, 0);
	const int cus = p.multiProcessorCount;
	printf("{\"cus\": %d, \"results\": [\n", cus);
	run_all<0>(out, cus);
	// occupancy sweep for a fast and a slow op
	for (int w : {1, 2, 4})
		run<1>(out, cus, w, false);
	for (int w : {1, 2, 4})
		run<6>(out, cus, w, w == 4);
	printf("]}\n");
	return 0;
}
