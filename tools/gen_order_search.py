#!/usr/bin/env python3
"""Generate tools/order_search.hip: an A/B of instruction orders for the
SHA-256 round (and the schedule word feeding it) on gfx950.

The kernels are bound by VALU issue and the issue cost of a
mixed stream depends on its order (tools/sha_variants.hip V6 vs V0: the same
instruction multiset, 5 % apart).  This tool enumerates orders of one
round's dataflow graph -- the 14 round instructions, plus for t >= 16 the 10
instructions of the schedule word W[t] -- as topological sorts chosen by
list scheduling under different priority rules, emits each as one asm block
per round (temporaries reused by liveness), and times them compute-only like
sha_variants.hip (17 blocks per lane, 16,384 waves, no memory traffic),
checking every variant's digests against a builtins reference.

Build: python3 tools/gen_order_search.py && hipcc --offload-arch=gfx950 -O3
-std=c++17 tools/order_search.hip -o tools/order_search
"""
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))

# op: (name, kind S/F, asm template, op sources)
ROUND = [
    ("r1", "S", "v_alignbit_b32 {r1}, {e}, {e}, 6", []),
    ("r2", "S", "v_alignbit_b32 {r2}, {e}, {e}, 11", []),
    ("r3", "S", "v_alignbit_b32 {r3}, {e}, {e}, 25", []),
    ("r4", "S", "v_alignbit_b32 {r4}, {a}, {a}, 2", []),
    ("r5", "S", "v_alignbit_b32 {r5}, {a}, {a}, 13", []),
    ("r6", "S", "v_alignbit_b32 {r6}, {a}, {a}, 22", []),
    ("x", "S", "v_add3_u32 {x}, {h}, {k}, {W}", ["WT"]),
    ("s1", "F", "v_bitop3_b32 {s1}, {r1}, {r2}, {r3} bitop3:0x96", ["r1", "r2", "r3"]),
    ("ch", "F", "v_bitop3_b32 {ch}, {e}, {f}, {g} bitop3:0xca", []),
    ("s0", "F", "v_bitop3_b32 {s0}, {r4}, {r5}, {r6} bitop3:0x96", ["r4", "r5", "r6"]),
    ("mj", "F", "v_bitop3_b32 {mj}, {a}, {b}, {c} bitop3:0xe8", []),
    ("t1", "S", "v_add3_u32 {t1}, {x}, {s1}, {ch}", ["x", "s1", "ch"]),
    ("D", "F", "v_add_u32 {d}, {d}, {t1}", ["t1"]),
    ("H", "S", "v_add3_u32 {h}, {t1}, {s0}, {mj}", ["t1", "s0", "mj", "x"]),
]
EXPAND = [
    ("q1", "S", "v_alignbit_b32 {q1}, {y2}, {y2}, 17", []),
    ("q2", "S", "v_alignbit_b32 {q2}, {y2}, {y2}, 19", []),
    ("q3", "S", "v_alignbit_b32 {q3}, {x15}, {x15}, 7", []),
    ("q4", "S", "v_alignbit_b32 {q4}, {x15}, {x15}, 18", []),
    ("q5", "F", "v_lshrrev_b32 {q5}, 10, {y2}", []),
    ("q6", "F", "v_lshrrev_b32 {q6}, 3, {x15}", []),
    ("p1", "F", "v_bitop3_b32 {p1}, {q1}, {q2}, {q5} bitop3:0x96", ["q1", "q2", "q5"]),
    ("p0", "F", "v_bitop3_b32 {p0}, {q3}, {q4}, {q6} bitop3:0x96", ["q3", "q4", "q6"]),
    ("u1", "S", "v_add3_u32 {w16}, {w16}, {p1}, {w7}", ["p1"]),
    ("WT", "F", "v_add_u32 {w16}, {w16}, {p0}", ["u1", "p0"]),
]
TEMPS = {"r1", "r2", "r3", "r4", "r5", "r6", "x", "s1", "ch", "s0", "mj", "t1",
         "q1", "q2", "q3", "q4", "q5", "q6", "p1", "p0"}
# the shipped kernel's order (sha2_device.h round256_asm / expand256_asm;
# h + K + W first, as the compiler places it before the asm block)
SHIPPED_R = ["x", "r1", "r2", "r3", "r4", "r5", "s1", "r6", "ch", "s0", "mj", "t1", "D", "H"]
SHIPPED_E = ["q1", "q2", "q3", "q4", "q5", "q6", "p1", "p0", "u1", "WT"] + SHIPPED_R


def graph(with_expand):
    ops = (EXPAND if with_expand else []) + ROUND
    names = {o[0] for o in ops}
    deps = {o[0]: [d for d in o[3] if d in names] for o in ops}
    return ops, deps


def depth_to_end(ops, deps):
    users = {o[0]: [] for o in ops}
    for n, ds in deps.items():
        for d in ds:
            users[d].append(n)
    memo = {}

    def f(n):
        if n not in memo:
            memo[n] = 1 + max((f(u) for u in users[n]), default=0)
        return memo[n]
    return {o[0]: f(o[0]) for o in ops}


def schedule(with_expand, rule, rng):
    ops, deps = graph(with_expand)
    kind = {o[0]: o[1] for o in ops}
    cp = depth_to_end(ops, deps)
    done, order = set(), []
    pri = {o[0]: rng.random() for o in ops}
    while len(order) < len(ops):
        ready = [o[0] for o in ops if o[0] not in done and all(d in done for d in deps[o[0]])]
        last = kind[order[-1]] if order else None
        if rule == "slow_first":
            key = lambda n: (kind[n] != "S", -cp[n], pri[n])
        elif rule == "fast_first":
            key = lambda n: (kind[n] != "F", -cp[n], pri[n])
        elif rule == "alternate":
            want = "F" if last == "S" else "S"
            key = lambda n: (kind[n] != want, -cp[n], pri[n])
        elif rule == "pairs":
            run = 0
            for m in reversed(order):
                if kind[m] != last:
                    break
                run += 1
            want = last if (order and run < 2) else ("F" if last == "S" else "S")
            key = lambda n: (kind[n] != want, -cp[n], pri[n])
        elif rule == "critical":
            key = lambda n: (-cp[n], pri[n])
        elif rule == "random":
            key = lambda n: pri[n]
        else:
            raise ValueError(rule)
        n = min(ready, key=key)
        order.append(n)
        done.add(n)
    return order


def alloc(order, with_expand):
    """Temporaries -> slots by liveness (a destination never shares a slot
    with a source of the same instruction)."""
    ops, deps = graph(with_expand)
    last_use = {}
    for i, n in enumerate(order):
        for d in deps[n]:
            last_use[d] = i
    free, slot, nslots = [], {}, 0
    for i, n in enumerate(order):
        if n in TEMPS:
            if free:
                slot[n] = free.pop(0)
            else:
                slot[n] = nslots
                nslots += 1
        for d in deps[n]:
            if d in TEMPS and last_use.get(d) == i:
                free.append(slot[d])
        free.sort()
    return slot, nslots


def emit_block(order, with_expand):
    ops, deps = graph(with_expand)
    pos = {n: i for i, n in enumerate(order)}
    assert sorted(order) == sorted(o[0] for o in ops)
    assert all(pos[d] < pos[n] for n in order for d in deps[n]), order
    tmpl = {o[0]: o[2] for o in ops}
    slot, nslots = alloc(order, with_expand)
    names = {n: f"%[t{slot[n]}]" for n in slot}
    names.update({v: f"%[{v}]" for v in ("a", "b", "c", "d", "e", "f", "g", "h", "k",
                                           "x15", "y2", "w7", "w16")})
    names["W"] = "%[w16]" if with_expand else "%[w]"
    return [tmpl[n].format(**names) for n in order], nslots


def asm_stmt(lines, n, with_expand):
    body = "".join(f'"{ln}\\n\\t"\n\t\t    ' for ln in lines)
    outs = ", ".join([f'[t{i}] "=&v"(t[{i}])' for i in range(n)] +
                     ['[h] "+v"(h)', '[d] "+v"(d)'] +
                     (['[w16] "+v"(w[T & 15])'] if with_expand else []))
    ins = ['[a] "v"(a)', '[b] "v"(b)', '[c] "v"(c)', '[e] "v"(e)', '[f] "v"(f)',
           '[g] "v"(g)', '[k] "s"(K256[T])']
    if with_expand:
        ins += ['[x15] "v"(w[(T - 15) & 15])', '[y2] "v"(w[(T - 2) & 15])',
                '[w7] "v"(w[(T - 7) & 15])']
    else:
        ins += ['[w] "v"(w[T & 15])']
    return (f'\t\t\tuint32_t t[{n}];\n\t\t\tasm({body.rstrip()}\n\t\t\t    : {outs}\n'
            f'\t\t\t    : {", ".join(ins)});\n')


def variant_struct(idx, label, o_r, o_e):
    lr, nr = emit_block(o_r, False)
    le, ne = emit_block(o_e, True)
    return f'''
// O{idx}: {label}
//   round : {" ".join(o_r)}
//   t>=16 : {" ".join(o_e)}
struct O{idx} {{
	template <int T> __device__ static void step(uint32_t (&s)[8], uint32_t (&w)[16]) {{
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		if (T < 16) {{
{asm_stmt(lr, nr, False)}		}} else {{
{asm_stmt(le, ne, True)}		}}
	}}
}};
'''


def variants():
    out = [("shipped order", SHIPPED_R, SHIPPED_E)]
    rules = [("slow_first", 1), ("fast_first", 1), ("alternate", 1), ("pairs", 1),
             ("critical", 1)] + [("random", s) for s in range(2, 12)] + \
            [("critical", s) for s in range(20, 23)] + [("alternate", s) for s in range(30, 33)] + \
            [("slow_first", s) for s in range(40, 43)]
    for rule, seed in rules:
        out.append((f"{rule} s{seed}", schedule(False, rule, random.Random(seed)),
                    schedule(True, rule, random.Random(seed))))
    return out


HEAD = r'''// GENERATED by tools/gen_order_search.py -- do not edit.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
#include <algorithm>

#define NBLK 17

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

__device__ __forceinline__ uint32_t rot(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

// Reference: builtins, the compiler's order.
struct REF {
	template <int T> __device__ static void step(uint32_t (&s)[8], uint32_t (&w)[16]) {
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		if (T >= 16) {
			uint32_t x = w[(T - 15) & 15], y = w[(T - 2) & 15];
			w[T & 15] += x3(rot(y, 17), rot(y, 19), y >> 10) + w[(T - 7) & 15] + x3(rot(x, 7), rot(x, 18), x >> 3);
		}
		uint32_t t1 = (h + K256[T] + w[T & 15]) + x3(rot(e, 6), rot(e, 11), rot(e, 25)) +
		    __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
		d += t1;
		h = t1 + x3(rot(a, 2), rot(a, 13), rot(a, 22)) + __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
	}
};
'''

TAIL = r'''
#ifndef FENCE
#define FENCE 2
#endif
template <class V, int T>
struct R {
	__device__ __forceinline__ static void run(uint32_t (&s)[8], uint32_t (&w)[16]) {
		V::template step<T>(s, w);
		if (FENCE > 0 && T % FENCE == FENCE - 1)
			__builtin_amdgcn_sched_barrier(0);
		R<V, T + 1>::run(s, w);
	}
};
template <class V>
struct R<V, 64> { __device__ __forceinline__ static void run(uint32_t (&)[8], uint32_t (&)[16]) {} };

template <class V>
__global__ __launch_bounds__(256) void kern(uint32_t *out, uint32_t seed)
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
'''


def main():
    vs = variants()
    parts = [HEAD]
    for i, (label, o_r, o_e) in enumerate(vs):
        parts.append(variant_struct(i, label, o_r, o_e))
    parts.append(TAIL)
    nv = len(vs) + 1
    names = ['"REF builtins"'] + [f'"O{i} {label}"' for i, (label, _, _) in enumerate(vs)]
    calls = ["\t\tbest[0] = std::min(best[0], timeit<REF>(out + 0 * n, blocks));"]
    calls += [f"\t\tbest[{i + 1}] = std::min(best[{i + 1}], timeit<O{i}>(out + {i + 1} * n, blocks));"
              for i in range(len(vs))]
    parts.append(f'''
int main()
{{
	const int blocks = 4096;  // 16384 waves
	const size_t n = (size_t)blocks * 256 * 8;
	const int NV = {nv};
	uint32_t *out;
	(void)hipMalloc(&out, n * 4 * NV);
	std::vector<uint32_t> ref(n), got(n);
	const char *names[] = {{{", ".join(names)}}};
	std::vector<float> best(NV, 1e9f);
	for (int i = 0; i < 30; i++) kern<REF><<<blocks, 256>>>(out, 7);  // clock ramp
	for (int round = 0; round < 3; round++) {{
{chr(10).join(calls)}
	}}
	(void)hipMemcpy(ref.data(), out, n * 4, hipMemcpyDeviceToHost);
	printf("{{\\"blocks_per_lane\\": %d, \\"waves\\": %d, \\"variants\\": [\\n", NBLK, blocks * 4);
	for (int v = 0; v < NV; v++) {{
		(void)hipMemcpy(got.data(), out + v * n, n * 4, hipMemcpyDeviceToHost);
		bool same = got == ref;
		printf("  {{\\"variant\\": \\"%s\\", \\"ms\\": %.4f, \\"same_as_REF\\": %s, \\"speedup_vs_REF\\": %.4f}}%s\\n",
		    names[v], best[v], same ? "true" : "false", best[0] / best[v], v == NV - 1 ? "" : ",");
	}}
	printf("]}}\\n");
	return 0;
}}
''')
    with open(os.path.join(HERE, "order_search.hip"), "w") as f:
        f.write("".join(parts))
    print(f"{len(vs)} variants")


if __name__ == "__main__":
    main()
