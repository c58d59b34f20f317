#!/usr/bin/env python3
"""Generate tools/bank_probe.hip: does the VGPR bank of an instruction's
sources change its issue cost on gfx950?

valu_probe.hip measured v_bitop3_b32 at 3.8 SIMD cycles per wave64
instruction with two loop-invariant sources and at 2.5 with sources taken
from neighbouring chain registers.  This probe pins every register (inline
asm on explicit VGPRs), so two rows differ only in the bank (register index
mod 4) of the sources.

Each kernel: 8 chains in v8..v15 (chain c writes v(8+c)), extra sources
in v16..v23, scratch v24..v55, a 1024-trip loop of 4 x 8 instructions, 8 waves/SIMD.
Build: python3 tools/gen_bank_probe.py && hipcc --offload-arch=gfx950 -O3
tools/bank_probe.hip -o tools/bank_probe
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
B = 8        # first chain register (v8..v55 used: < 64 VGPRs, 8 waves/SIMD)


def pat_srcs(pat, c):
    if pat == 3:    # three banks: c, c+1, c+2
        return B + (c + 1) % 8, B + (c + 2) % 8
    if pat == 1:    # one bank: c, c, c
        return B + (c + 4) % 8, B + 8 + c
    if pat == 2:    # two banks: c, c, c+1
        return B + (c + 4) % 8, B + 8 + (c + 1) % 8
    raise ValueError(pat)


# (name, template over d, a, b, pattern)
ROWS = [
    ("v_bitop3_b32 xor3, srcs in 3 banks", "v_bitop3_b32 v{d}, v{d}, v{a}, v{b} bitop3:0x96", 3),
    ("v_bitop3_b32 xor3, srcs in 2 banks", "v_bitop3_b32 v{d}, v{d}, v{a}, v{b} bitop3:0x96", 2),
    ("v_bitop3_b32 xor3, srcs in 1 bank", "v_bitop3_b32 v{d}, v{d}, v{a}, v{b} bitop3:0x96", 1),
    ("v_bitop3_b32 ch, srcs in 3 banks", "v_bitop3_b32 v{d}, v{d}, v{a}, v{b} bitop3:0xca", 3),
    ("v_bitop3_b32 ch, srcs in 1 bank", "v_bitop3_b32 v{d}, v{d}, v{a}, v{b} bitop3:0xca", 1),
    ("v_add3_u32, srcs in 3 banks", "v_add3_u32 v{d}, v{d}, v{a}, v{b}", 3),
    ("v_add3_u32, srcs in 2 banks", "v_add3_u32 v{d}, v{d}, v{a}, v{b}", 2),
    ("v_add3_u32, srcs in 1 bank", "v_add3_u32 v{d}, v{d}, v{a}, v{b}", 1),
    ("v_alignbit_b32 x,y,7, srcs in 2 banks", "v_alignbit_b32 v{d}, v{d}, v{a}, 7", 3),
    ("v_alignbit_b32 x,y,7, srcs in 1 bank", "v_alignbit_b32 v{d}, v{d}, v{a}, 7", 1),
    ("v_alignbit_b32 x,x,7 (rotate)", "v_alignbit_b32 v{d}, v{d}, v{d}, 7", 3),
    ("v_alignbit_b32 y,y,7 (rotate of other chain)", "v_alignbit_b32 v{d}, v{a}, v{a}, 7", 3),
    ("v_add_u32 v,v, srcs in 2 banks", "v_add_u32 v{d}, v{d}, v{a}", 3),
    ("v_add_u32 v,v, srcs in 1 bank", "v_add_u32 v{d}, v{d}, v{a}", 1),
    ("v_xor_b32 v,v, srcs in 2 banks", "v_xor_b32 v{d}, v{d}, v{a}", 3),
    ("v_xor_b32 v,v, srcs in 1 bank", "v_xor_b32 v{d}, v{d}, v{a}", 1),
    ("v_lshrrev_b32 7,v (other chain)", "v_lshrrev_b32 v{d}, 7, v{a}", 3),
    ("v_lshlrev_b32 7,v (other chain)", "v_lshlrev_b32 v{d}, 7, v{a}", 3),
    ("v_perm_b32 x,y,s, srcs in 2 banks", "v_perm_b32 v{d}, v{d}, v{a}, s40", 3),
    ("v_lshl_add_u32 x,7,y (2 banks)", "v_lshl_add_u32 v{d}, v{d}, 7, v{a}", 3),
    ("v_add_u32 literal (K)", "v_add_u32 v{d}, 0x428a2f98, v{d}", 3),
    # SHA-256 round-shaped mixes: rotate triple + xor3, and add3 chains
    ("mix: 3 rot + bitop3 (Sigma), 3-bank", None, 3),
    ("mix: 3 rot + bitop3 (Sigma), 1-bank", None, 1),
    ("mix: bitop3 + add_u32 alternating, 3-bank", None, 3),
]
# Slow/fast sequence rows: S = v_alignbit_b32 rotate, F = v_xor_b32; the
# string is one wave's instruction order, chains taken round-robin.
SEQS = ["SF", "SSFF", "SSSSFFFF", "SSF", "SSSF", "SSSSSSFF", "SFF", "SFFF",
        "S", "F", "SSSSSSSS" + "FFFFFFFF"]
ROWS += [("seq " + q, "SEQ:" + q, 3) for q in SEQS]
# Split rows: two kinds of wave on the same CU, each running a pure stream;
# by workgroup parity the two kinds share every SIMD, by wave parity they
# (likely) land on different SIMDs.
ROWS += [("split by workgroup: S-only | F-only waves", "SPLITB:S|F", 3),
         ("split by wave: S-only | F-only waves", "SPLITW:S|F", 3),
         ("split by workgroup: SF | SF (control)", "SPLITB:SF|SF", 3)]


def instrs(i, name, tmpl, pat):
    out = []
    for c in range(8):
        d = B + c
        a, b = pat_srcs(pat, c)
        if tmpl is not None:
            out.append(tmpl.format(d=d, a=a, b=b))
        elif name.startswith("mix: 3 rot"):
            # Sigma-shaped: three rotates of another chain's register, xor3.
            # Scratch v(B+16+4c)..v(B+19+4c) holds one register per bank.
            r2 = B + 16 + 4 * c + (c + 1) % 4
            r3 = B + 16 + 4 * c + (c + 2) % 4 if pat == 3 else B + 8 + c
            if pat == 1:
                r2 = B + 16 + 4 * c + c % 4
            out.append(f"v_alignbit_b32 v{d}, v{a}, v{a}, 6")
            out.append(f"v_alignbit_b32 v{r2}, v{a}, v{a}, 11")
            out.append(f"v_alignbit_b32 v{r3}, v{a}, v{a}, 25")
            out.append(f"v_bitop3_b32 v{d}, v{d}, v{r2}, v{r3} bitop3:0x96")
        else:
            out.append(f"v_bitop3_b32 v{d}, v{d}, v{a}, v{b} bitop3:0x96" if c % 2
                       else f"v_add_u32 v{d}, v{d}, v{a}")
    return out


def seq_instrs(q):
    """len(q) * 8 instructions following pattern q, chain c = i mod 8."""
    out = []
    for i in range(len(q) * 8):
        c = i % 8
        d, a = B + c, B + (c + 1) % 8
        if q[i % len(q)] == "S":
            out.append(f"v_alignbit_b32 v{d}, v{d}, v{d}, 7")
        else:
            out.append(f"v_xor_b32 v{d}, v{d}, v{a}")
    return out


def kernel(i, name, tmpl, pat):
    if tmpl and tmpl.startswith("SPLIT"):
        return split_kernel(i, tmpl)
    body = (seq_instrs(tmpl[4:]) if tmpl and tmpl.startswith("SEQ:")
            else instrs(i, name, tmpl, pat))
    n = len(body)
    loop = "".join(f'"{s}\\n\\t"\n\t    ' for s in body) * 4
    init = "".join(
        f'"v_add_u32 v{r}, {r - B}, %1\\n\\t"\n\t    ' for r in range(B, B + 48))
    return f'''
__global__ __launch_bounds__(256) void k{i}(uint32_t *out, uint32_t seed)
{{
	uint64_t t0 = __builtin_amdgcn_s_memtime();
	uint32_t x, v0 = threadIdx.x ^ seed;
	asm volatile(
	    {init}"s_mov_b32 s40, %2\\n\\t"
	    "s_movk_i32 s41, 0x400\\n"
	    "1:\\n\\t"
	    {loop}"s_sub_u32 s41, s41, 1\\n\\t"
	    "s_cmp_lg_u32 s41, 0\\n\\t"
	    "s_cbranch_scc1 1b\\n\\t"
	    "v_xor_b32 %0, v8, v9\\n\\t"
	    "v_bitop3_b32 %0, %0, v10, v11 bitop3:0x96\\n\\t"
	    "v_bitop3_b32 %0, %0, v12, v13 bitop3:0x96\\n\\t"
	    "v_bitop3_b32 %0, %0, v14, v15 bitop3:0x96\\n\\t"
	    "v_bitop3_b32 %0, %0, v16, v17 bitop3:0x96\\n\\t"
	    "v_bitop3_b32 %0, %0, v24, v28 bitop3:0x96"
	    : "=v"(x)
	    : "v"(v0), "s"(seed)
	    : {", ".join(f'"v{r}"' for r in range(B, B + 48))}, "s40", "s41", "scc");
	if (x == 0x12345678u)
		out[0] = x;
	uint64_t t1 = __builtin_amdgcn_s_memtime();
	if ((threadIdx.x & 63) == 0)
		out[16 + blockIdx.x * 4 + threadIdx.x / 64] = (uint32_t)(t1 - t0);
}}
static const int kN{i} = {n * 4};	/* instructions per loop trip */
'''


def split_kernel(i, tmpl):
    """Two asm loops selected per wave (uniform branch): pattern qa for
    workgroups (SPLITB) or waves (SPLITW) of even parity, qb for odd."""
    kind, pats = tmpl.split(":")
    qa, qb = pats.split("|")
    assert len(qa) == len(qb)
    sel = "(blockIdx.x & 1)" if kind == "SPLITB" else "((threadIdx.x >> 6) & 1)"
    clob = ", ".join(f'"v{r}"' for r in range(B, B + 48))
    init = "".join(
        f'"v_add_u32 v{r}, {r - B}, %1\\n\\t"\n\t    ' for r in range(B, B + 48))

    def block(q):
        loop = "".join(f'"{x}\\n\\t"\n\t    ' for x in seq_instrs(q)) * 4
        return f'''asm volatile(
	    {init}"s_movk_i32 s41, 0x400\\n"
	    "1:\\n\\t"
	    {loop}"s_sub_u32 s41, s41, 1\\n\\t"
	    "s_cmp_lg_u32 s41, 0\\n\\t"
	    "s_cbranch_scc1 1b\\n\\t"
	    "v_xor_b32 %0, v8, v9\\n\\t"
	    "v_bitop3_b32 %0, %0, v10, v11 bitop3:0x96\\n\\t"
	    "v_bitop3_b32 %0, %0, v12, v13 bitop3:0x96\\n\\t"
	    "v_bitop3_b32 %0, %0, v14, v15 bitop3:0x96"
	    : "=v"(x)
	    : "v"(v0)
	    : {clob}, "s41", "scc");'''
    return f'''
__global__ __launch_bounds__(256) void k{i}(uint32_t *out, uint32_t seed)
{{
	uint32_t x, v0 = threadIdx.x ^ seed;
	if (__builtin_amdgcn_readfirstlane({sel}) == 0) {{
		{block(qa)}
	}} else {{
		{block(qb)}
	}}
	if (x == 0x12345678u)
		out[0] = x;
}}
static const int kN{i} = {len(qa) * 8 * 4};	/* instructions per loop trip */
'''


def main():
    parts = ["""// GENERATED by tools/gen_bank_probe.py -- do not edit.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define TRIPS 1024
"""]
    for i, (name, tmpl, pat) in enumerate(ROWS):
        parts.append(kernel(i, name, tmpl, pat))
    parts.append("""
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

static void report(const char *name, int cus, float ms, int per_trip, bool last)
{
	const int blocks = cus * 8;
	double instr = (double)blocks * 4 * TRIPS * per_trip;
	double cyc = ms * 1e-3 * 2.4e9 * cus * 4 / instr;
	printf("  {\\"op\\": \\"%s\\", \\"ms\\": %.4f, \\"simd_cycles_per_wave_instr_at_2.4GHz\\": %.3f}%s\\n",
	    name, ms, cyc, last ? "" : ",");
}

int main()
{
	uint32_t *out;
	(void)hipMalloc(&out, sizeof(uint32_t) * (16 + 256 * 8 * 4));
	hipDeviceProp_t p;
	(void)hipGetDeviceProperties(&p, 0);
	const int cus = p.multiProcessorCount;
	// clock ramp
	for (int i = 0; i < 20; i++)
		k0<<<cus * 8, 256>>>(out, 1);
	(void)hipDeviceSynchronize();
	printf("{\\"cus\\": %d, \\"waves_per_simd\\": 8, \\"results\\": [\\n", cus);
""")
    for i, (name, _, _) in enumerate(ROWS):
        parts.append(
            f'\treport("{name}", cus, time_kernel([&] {{ k{i}<<<cus * 8, 256>>>(out, 1); }}), '
            f'kN{i}, {"true" if i == len(ROWS) - 1 else "false"});\n')
    parts.append("\tprintf(\"]}\\n\");\n\treturn 0;\n}\n")
    with open(os.path.join(HERE, "bank_probe.hip"), "w") as f:
        f.write("".join(parts))


if __name__ == "__main__":
    main()
