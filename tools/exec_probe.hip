// Does a VALU instruction cost less when EXEC has whole 16-lane groups off?
// (tools/exec_probe.hip; `make -C tools exec_probe`; gpu: tools/exec_probe)
//
// One asm loop of 64 VALU instructions per trip, either 8 independent
// chains (issue-bound) or one dependent chain (latency-bound), of a
// full-rate (v_xor_b32) or half-rate (v_alignbit_b32) op, run under an
// EXEC mask chosen per lane: all 64 lanes, lanes 0-31, lanes 0-15 (one
// 16-lane group), lane 0 alone, or one lane in each 16-lane group.
// A lone wave (grid of one) gives the single-wave issue / latency cost,
// 8 waves per SIMD over the whole chip the throughput cost.  Cycles come
// from s_memtime around the loop (lone wave) and from hipEvents (grid).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define TRIPS 4096

#define X8(s) s s s s s s s s
// 8 independent chains, v40..v47
#define IND_XOR "v_xor_b32 v40, v40, v48\n\tv_xor_b32 v41, v41, v48\n\t" \
	"v_xor_b32 v42, v42, v48\n\tv_xor_b32 v43, v43, v48\n\t" \
	"v_xor_b32 v44, v44, v48\n\tv_xor_b32 v45, v45, v48\n\t" \
	"v_xor_b32 v46, v46, v48\n\tv_xor_b32 v47, v47, v48\n\t"
#define IND_ALN "v_alignbit_b32 v40, v40, v40, 7\n\tv_alignbit_b32 v41, v41, v41, 7\n\t" \
	"v_alignbit_b32 v42, v42, v42, 7\n\tv_alignbit_b32 v43, v43, v43, 7\n\t" \
	"v_alignbit_b32 v44, v44, v44, 7\n\tv_alignbit_b32 v45, v45, v45, 7\n\t" \
	"v_alignbit_b32 v46, v46, v46, 7\n\tv_alignbit_b32 v47, v47, v47, 7\n\t"
// one dependent chain
#define DEP_XOR "v_xor_b32 v40, v40, v48\n\tv_xor_b32 v40, v40, v49\n\t" \
	"v_xor_b32 v40, v40, v48\n\tv_xor_b32 v40, v40, v49\n\t" \
	"v_xor_b32 v40, v40, v48\n\tv_xor_b32 v40, v40, v49\n\t" \
	"v_xor_b32 v40, v40, v48\n\tv_xor_b32 v40, v40, v49\n\t"
#define DEP_ALN "v_alignbit_b32 v40, v40, v40, 7\n\tv_alignbit_b32 v40, v40, v40, 9\n\t" \
	"v_alignbit_b32 v40, v40, v40, 7\n\tv_alignbit_b32 v40, v40, v40, 9\n\t" \
	"v_alignbit_b32 v40, v40, v40, 7\n\tv_alignbit_b32 v40, v40, v40, 9\n\t" \
	"v_alignbit_b32 v40, v40, v40, 7\n\tv_alignbit_b32 v40, v40, v40, 9\n\t"
// SHA-like mix: 3 rotates + 1 xor3 per 4, 2 chains interleaved
#define MIX "v_alignbit_b32 v41, v40, v40, 6\n\tv_alignbit_b32 v42, v40, v40, 11\n\t" \
	"v_alignbit_b32 v43, v40, v40, 25\n\tv_bitop3_b32 v40, v41, v42, v43 bitop3:0x96\n\t" \
	"v_alignbit_b32 v45, v44, v44, 2\n\tv_alignbit_b32 v46, v44, v44, 13\n\t" \
	"v_alignbit_b32 v47, v44, v44, 22\n\tv_bitop3_b32 v44, v45, v46, v47 bitop3:0x96\n\t"

#define BODY(k) X8(k)	/* 64 instructions */

#define KERNEL(name, body)                                                    \
__global__ __launch_bounds__(64) void name(uint32_t *out, int mask, uint32_t seed) \
{                                                                             \
	const uint32_t lane = threadIdx.x;                                    \
	bool act = mask == 0 ? true : mask == 1 ? lane < 32 : mask == 2 ?     \
	    lane < 16 : mask == 3 ? lane == 0 : (lane & 15) == 0;              \
	uint32_t x = lane ^ seed;                                             \
	uint64_t t0 = 0, t1 = 0;                                              \
	if (act) {                                                            \
		t0 = __builtin_amdgcn_s_memtime();                            \
		asm volatile(                                                 \
		    "v_mov_b32 v40, %1\n\tv_mov_b32 v41, %1\n\t"              \
		    "v_mov_b32 v42, %1\n\tv_mov_b32 v43, %1\n\t"              \
		    "v_mov_b32 v44, %1\n\tv_mov_b32 v45, %1\n\t"              \
		    "v_mov_b32 v46, %1\n\tv_mov_b32 v47, %1\n\t"              \
		    "v_mov_b32 v48, %1\n\tv_not_b32 v49, %1\n\t"              \
		    "s_movk_i32 s41, %2\n"                                    \
		    "1:\n\t" BODY(body)                                       \
		    "s_sub_u32 s41, s41, 1\n\t"                               \
		    "s_cmp_lg_u32 s41, 0\n\t"                                 \
		    "s_cbranch_scc1 1b\n\t"                                   \
		    "v_xor_b32 %0, v40, v41\n\t"                              \
		    "v_bitop3_b32 %0, %0, v42, v43 bitop3:0x96\n\t"           \
		    "v_bitop3_b32 %0, %0, v44, v45 bitop3:0x96\n\t"           \
		    "v_bitop3_b32 %0, %0, v46, v47 bitop3:0x96"               \
		    : "=v"(x)                                                 \
		    : "v"(x), "i"(TRIPS)                                      \
		    : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", \
		      "v48", "v49", "s41", "scc");                            \
		t1 = __builtin_amdgcn_s_memtime();                            \
	}                                                                     \
	if (x == 0x12345678u)                                                 \
		out[1] = x;                                                   \
	if (lane == 0)                                                        \
		out[2 + blockIdx.x] = (uint32_t)(t1 - t0);                    \
}

KERNEL(k_ind_xor, IND_XOR)
KERNEL(k_ind_aln, IND_ALN)
KERNEL(k_dep_xor, DEP_XOR)
KERNEL(k_dep_aln, DEP_ALN)
KERNEL(k_mix, MIX)

typedef void (*kfn)(uint32_t *, int, uint32_t);

int main()
{
	hipDeviceProp_t p;
	(void)hipGetDeviceProperties(&p, 0);
	const int cus = p.multiProcessorCount;
	const int grid_full = cus * 4 * 8;	/* 8 waves per SIMD */
	uint32_t *out;
	(void)hipMalloc(&out, sizeof(uint32_t) * (2 + grid_full));
	uint32_t *h = new uint32_t[2 + grid_full];
	struct { const char *name; kfn f; } ks[] = {
		{"8 independent v_xor_b32", k_ind_xor},
		{"8 independent v_alignbit_b32", k_ind_aln},
		{"dependent v_xor_b32", k_dep_xor},
		{"dependent v_alignbit_b32", k_dep_aln},
		{"2 Sigma chains (3 alignbit + xor3)", k_mix},
	};
	const char *masks[] = {"64 lanes", "lanes 0-31", "lanes 0-15", "lane 0",
	    "lanes 0,16,32,48"};
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	/* clock ramp */
	for (int i = 0; i < 30; i++)
		k_ind_xor<<<grid_full, 64>>>(out, 0, 1);
	(void)hipDeviceSynchronize();
	printf("{\"cus\": %d, \"instr_per_wave\": %d, \"rows\": [\n", cus, TRIPS * 64);
	bool first = true;
	for (auto &k : ks) {
		for (int m = 0; m < 5; m++) {
			/* lone wave: s_memtime cycles per instruction */
			k.f<<<1, 64>>>(out, m, 1);
			(void)hipDeviceSynchronize();
			k.f<<<1, 64>>>(out, m, 2);
			(void)hipMemcpy(h, out, sizeof(uint32_t) * 3, hipMemcpyDeviceToHost);
			const double lone = (double)h[2] / (TRIPS * 64.0);
			/* full grid, 8 waves per SIMD: event time */
			k.f<<<grid_full, 64>>>(out, m, 3);
			(void)hipEventRecord(a);
			for (int r = 0; r < 3; r++)
				k.f<<<grid_full, 64>>>(out, m, 4 + r);
			(void)hipEventRecord(b);
			(void)hipEventSynchronize(b);
			float ms;
			(void)hipEventElapsedTime(&ms, a, b);
			ms /= 3;
			/* SIMD cycles per wave instruction at 2.4 GHz */
			const double grid = ms * 1e-3 * 2.4e9 * cus * 4 /
			    ((double)grid_full * TRIPS * 64);
			printf("%s  {\"op\": \"%s\", \"exec\": \"%s\", "
			    "\"lone_wave_memtime_cycles_per_instr\": %.3f, "
			    "\"grid_8waves_simd_cycles_per_instr\": %.3f, \"grid_ms\": %.4f}",
			    first ? "" : ",\n", k.name, masks[m], lone, grid, ms);
			first = false;
		}
	}
	printf("\n]}\n");
	return 0;
}
