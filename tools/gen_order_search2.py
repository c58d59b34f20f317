#!/usr/bin/env python3
"""Generate tools/order_search2.hip: SHA-256 instruction orders over TWO
rounds (and their two schedule words) per asm block.

tools/bank_probe (profiles/round1/valu_bank_seq_probe.json) found that in a
stream mixing half-rate (v_alignbit, v_add3) and full-rate (v_bitop3,
v_add, v_lshrrev) instructions every instruction issues at ~4 SIMD cycles,
unless the full-rate ones come in long runs (8 slow then 8 fast per wave:
3.87 against 4.05-4.14 for shorter runs).  One round's dependencies allow
runs of at most ~4; two rounds plus two independent schedule words allow
longer ones.  Same harness as tools/gen_order_search.py.
"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_order_search as g1  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

# register roles of round 1 in terms of round 0's operands (the state
# renaming of one round: a1 = h0 (new a), e1 = d0 (new e), ...)
ROLE1 = {"a": "h", "b": "a", "c": "b", "d": "c", "e": "d", "f": "e", "g": "f", "h": "g"}


def block_ops(with_expand):
    ops = []   # (name, kind, template, deps)
    for j in (0, 1):
        if with_expand:
            for n, k, t, d in g1.EXPAND:
                t = t.replace("{x15}", "{x15_%d}" % j).replace("{y2}", "{y2_%d}" % j) \
                     .replace("{w7}", "{w7_%d}" % j).replace("{w16}", "{w16_%d}" % j)
                for q in ("q1", "q2", "q3", "q4", "q5", "q6", "p1", "p0"):
                    t = t.replace("{%s}" % q, "{%s_%d}" % (q, j))
                ops.append((f"{n}_{j}E", k, t, [f"{x}_{j}E" for x in d]))
        for n, k, t, d in g1.ROUND:
            if j == 1:
                # rename state roles (longest names first is not needed: single letters in braces)
                t = "".join(t)
                for role in "abcdefgh":
                    t = t.replace("{%s}" % role, "{R1_%s}" % role)
                for role, src in ROLE1.items():
                    t = t.replace("{R1_%s}" % role, "{%s}" % src)
            t = t.replace("{k}", "{k_%d}" % j).replace("{W}", "{W_%d}" % j)
            for q in ("r1", "r2", "r3", "r4", "r5", "r6", "x", "s1", "ch", "s0", "mj", "t1"):
                t = t.replace("{%s}" % q, "{%s_%d}" % (q, j))
            deps = [f"{x}_{j}" if x != "WT" else f"WT_{j}E" for x in d]
            if not with_expand:
                deps = [x for x in deps if not x.endswith("E")]
            ops.append((f"{n}_{j}", k, t, deps))
    # cross-round dependencies: round 1 reads a1 = h (after H_0), e1 = d
    # (after D_0); it writes c (D_1) and g (H_1), which round 0 reads.
    extra = {}
    for n, k, t, d in ops:
        if n.endswith("_1"):
            if "{h}" in t and n != "H_1":
                extra.setdefault(n, []).append("H_0")
            if "{d}" in t and n != "D_1":
                extra.setdefault(n, []).append("D_0")
    extra.setdefault("D_1", []).extend(["mj_0"])
    extra.setdefault("H_1", []).extend(["ch_0", "x_1"])
    out = []
    for n, k, t, d in ops:
        out.append((n, k, t, d + extra.get(n, [])))
    return out


def schedule(ops, rule, rng):
    deps = {o[0]: o[3] for o in ops}
    kind = {o[0]: o[1] for o in ops}
    users = {o[0]: [] for o in ops}
    for n, ds in deps.items():
        for d in ds:
            users[d].append(n)
    memo = {}

    def cp(n):
        if n not in memo:
            memo[n] = 1 + max((cp(u) for u in users[n]), default=0)
        return memo[n]
    pri = {o[0]: rng.random() for o in ops}
    done, order = set(), []
    while len(order) < len(ops):
        ready = [o[0] for o in ops if o[0] not in done and all(d in done for d in deps[o[0]])]
        last = kind[order[-1]] if order else "S"
        if rule == "runs":
            key = lambda n: (kind[n] != last, -cp(n), pri[n])
        elif rule == "runs_rand":
            key = lambda n: (kind[n] != last, pri[n])
        elif rule == "slow_first":
            key = lambda n: (kind[n] != "S", -cp(n), pri[n])
        elif rule == "fast_first":
            key = lambda n: (kind[n] != "F", -cp(n), pri[n])
        elif rule == "critical":
            key = lambda n: (-cp(n), pri[n])
        else:
            raise ValueError(rule)
        n = min(ready, key=key)
        order.append(n)
        done.add(n)
    return order


def emit(ops, order):
    deps = {o[0]: o[3] for o in ops}
    tmpl = {o[0]: o[2] for o in ops}
    pos = {n: i for i, n in enumerate(order)}
    assert all(pos[d] < pos[n] for n in order for d in deps[n])
    # temporaries: every op except the in-place writers
    inplace = {"D_0", "H_0", "D_1", "H_1", "u1_0E", "WT_0E", "u1_1E", "WT_1E"}
    last_use = {}
    for i, n in enumerate(order):
        for d in deps[n]:
            last_use[d] = i
    free, slot, ns = [], {}, 0
    for i, n in enumerate(order):
        if n not in inplace:
            slot[n] = free.pop(0) if free else ns
            if slot[n] == ns:
                ns += 1
        for d in deps[n]:
            if d in slot and last_use.get(d) == i:
                free.append(slot[d])
        free.sort()
    names = {}
    for n, s in slot.items():
        base = n.split("_")[0]
        j = n.split("_")[1][0]
        names[f"{base}_{j}"] = f"%[t{s}]"
    for v in ("a", "b", "c", "d", "e", "f", "g", "h", "k_0", "k_1", "W_0", "W_1",
              "x15_0", "y2_0", "w7_0", "w16_0", "x15_1", "y2_1", "w7_1", "w16_1"):
        names[v] = f"%[{v}]"
    lines = [tmpl[n].format(**names) for n in order]
    return lines, ns


def asm_stmt(lines, n, with_expand):
    body = "".join(f'"{ln}\\n\\t"\n\t\t    ' for ln in lines)
    outs = [f'[t{i}] "=&v"(t[{i}])' for i in range(n)] + \
        ['[h] "+v"(h)', '[d] "+v"(d)', '[c] "+v"(c)', '[g] "+v"(g)']
    ins = ['[a] "v"(a)', '[b] "v"(b)', '[e] "v"(e)', '[f] "v"(f)',
           '[k_0] "s"(K256[T])', '[k_1] "s"(K256[T + 1])']
    if with_expand:
        outs += ['[w16_0] "+v"(w[T & 15])', '[w16_1] "+v"(w[(T + 1) & 15])']
        ins += ['[x15_0] "v"(w[(T - 15) & 15])', '[y2_0] "v"(w[(T - 2) & 15])',
                '[w7_0] "v"(w[(T - 7) & 15])', '[x15_1] "v"(w[(T - 14) & 15])',
                '[y2_1] "v"(w[(T - 1) & 15])', '[w7_1] "v"(w[(T - 6) & 15])']
        body = body.replace("%[W_0]", "%[w16_0]").replace("%[W_1]", "%[w16_1]")
    else:
        ins += ['[W_0] "v"(w[T & 15])', '[W_1] "v"(w[(T + 1) & 15])']
    return (f'\t\t\tuint32_t t[{n}];\n\t\t\tasm({body.rstrip()}\n\t\t\t    : {", ".join(outs)}\n'
            f'\t\t\t    : {", ".join(ins)});\n')


def variant(idx, rule, seed):
    res = []
    for we in (False, True):
        ops = block_ops(we)
        order = schedule(ops, rule, random.Random(seed))
        lines, n = emit(ops, order)
        kinds = "".join({o[0]: o[1] for o in ops}[x] for x in order)
        res.append((lines, n, kinds))
    return f'''
// P{idx}: {rule} s{seed}
//   t<16 kinds : {res[0][2]}
//   t>=16 kinds: {res[1][2]}
struct P{idx} {{
	template <int T> __device__ static void step(uint32_t (&s)[8], uint32_t (&w)[16]) {{
		uint32_t &a = s[(0 - T) & 7], &b = s[(1 - T) & 7], &c = s[(2 - T) & 7];
		uint32_t &d = s[(3 - T) & 7], &e = s[(4 - T) & 7], &f = s[(5 - T) & 7];
		uint32_t &g = s[(6 - T) & 7], &h = s[(7 - T) & 7];
		if (T < 16) {{
{asm_stmt(res[0][0], res[0][1], False)}		}} else {{
{asm_stmt(res[1][0], res[1][1], True)}		}}
	}}
}};
'''


VARIANTS = [("runs", 1), ("runs", 2), ("runs", 3), ("runs_rand", 4), ("runs_rand", 5),
            ("runs_rand", 6), ("slow_first", 1), ("slow_first", 7), ("fast_first", 1),
            ("critical", 1), ("critical", 8)]

TAIL2 = g1.TAIL.replace("V::template step<T>(s, w);\n\t\tif (FENCE > 0 && T % FENCE == FENCE - 1)\n\t\t\t__builtin_amdgcn_sched_barrier(0);\n\t\tR<V, T + 1>::run(s, w);",
                        "V::template step<T>(s, w);\n\t\t__builtin_amdgcn_sched_barrier(0);\n\t\tR<V, T + 2>::run(s, w);")


def main():
    assert TAIL2 != g1.TAIL
    parts = [g1.HEAD]
    # O0 of the one-round search (the shipped order) as the in-process baseline
    parts.append(g1.variant_struct(0, "shipped order", g1.SHIPPED_R, g1.SHIPPED_E))
    for i, (rule, seed) in enumerate(VARIANTS):
        parts.append(variant(i, rule, seed))
    parts.append(g1.TAIL.replace("struct R {", "struct R1 {").replace("R<V, T + 1>", "R1<V, T + 1>")
                 .replace("struct R<V, 64>", "struct R1<V, 64>").replace("template <class V>\n__global__", "template <class V, bool TWO>\n__global__")
                 .replace("R<V, 0>::run(s, w);", "if (TWO) R2<V, 0>::run(s, w); else R1<V, 0>::run(s, w);")
                 .replace("kern<V><<<", "kern<V, TWO><<<").replace("template <class V>\nstatic float timeit", "template <class V, bool TWO>\nstatic float timeit")
                 .replace("template <class V, int T>\nstruct R1 {",
                          "template <class V, int T>\nstruct R2 {\n\t__device__ __forceinline__ static void run(uint32_t (&s)[8], uint32_t (&w)[16]) {\n\t\tV::template step<T>(s, w);\n\t\t__builtin_amdgcn_sched_barrier(0);\n\t\tR2<V, T + 2>::run(s, w);\n\t}\n};\ntemplate <class V>\nstruct R2<V, 64> { __device__ __forceinline__ static void run(uint32_t (&)[8], uint32_t (&)[16]) {} };\n\ntemplate <class V, int T>\nstruct R1 {"))
    nv = len(VARIANTS) + 2
    names = ['"REF builtins"', '"O0 shipped order (1 round/block)"'] + \
        [f'"P{i} {r} s{s} (2 rounds/block)"' for i, (r, s) in enumerate(VARIANTS)]
    calls = ["\t\tbest[0] = std::min(best[0], timeit<REF, false>(out + 0 * n, blocks));",
             "\t\tbest[1] = std::min(best[1], timeit<O0, false>(out + 1 * n, blocks));"]
    calls += [f"\t\tbest[{i + 2}] = std::min(best[{i + 2}], timeit<P{i}, true>(out + {i + 2} * n, blocks));"
              for i in range(len(VARIANTS))]
    main_src = f'''
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
	for (int i = 0; i < 30; i++) kern<REF, false><<<blocks, 256>>>(out, 7);  // clock ramp
	for (int round = 0; round < 3; round++) {{
{chr(10).join(calls)}
	}}
	(void)hipMemcpy(ref.data(), out, n * 4, hipMemcpyDeviceToHost);
	printf("{{\\"blocks_per_lane\\": %d, \\"waves\\": %d, \\"variants\\": [\\n", NBLK, blocks * 4);
	for (int v = 0; v < NV; v++) {{
		(void)hipMemcpy(got.data(), out + v * n, n * 4, hipMemcpyDeviceToHost);
		bool same = got == ref;
		printf("  {{\\"variant\\": \\"%s\\", \\"ms\\": %.4f, \\"same_as_REF\\": %s, \\"speedup_vs_O0\\": %.4f}}%s\\n",
		    names[v], best[v], same ? "true" : "false", best[1] / best[v], v == NV - 1 ? "" : ",");
	}}
	printf("]}}\\n");
	return 0;
}}
'''
    parts.append(main_src)
    with open(os.path.join(HERE, "order_search2.hip"), "w") as f:
        f.write("".join(parts))
    print(len(VARIANTS), "variants")


if __name__ == "__main__":
    main()
