#!/usr/bin/env python3
"""VALU issue floor of the shipped kernels, from their gfx950 ISA.

The SHA kernels are bound by vector-instruction issue, not by HBM (DESIGN.md
5.3).  Their floor is therefore a sum over the instructions a wave issues of
what each one costs the SIMD.  This tool:

  1. reads the device assembly of sha2_kernels.hip (`make -C
     ilias_net2_amd/csrc asm` writes ilias_net2_amd/csrc/build/sha2_kernels.s),
  2. for each bench config's kernel, counts the VALU instructions of its
     innermost loop body (the block loop: >94 % of the instructions a C2/C4
     wave issues) by mnemonic and operand form,
  3. prices them: every instruction of a loop that mixes half-rate
     (v_alignbit, v_add3, v_perm, v_lshl_add_u64, ...) and full-rate
     (v_bitop3, v_add, v_xor, v_lshrrev, ...) instructions at the measured
     cost of such a stream (profiles/round1/valu_bank_seq_probe.json, row
     "mix: 3 rot + bitop3 (Sigma)": 3.95 SIMD cycles per wave64 instruction
     at 2.4 GHz, 8 waves/SIMD).  The probe's sequence rows show why: in a
     mixed stream every instruction issues at ~4 cycles, whatever its
     class (S F S F 4.11, S F F F 4.09, 8 S then 8 F 3.87; pure full-rate
     2.44, pure half-rate 4.21).  The additive price (each instruction at
     its own pure-stream cost, profiles/round1/valu_probe.json) is kept
     alongside as the optimistic bound,
  4. writes profiles/isa_mix.json: per config, the loop's instruction mix and
     its mean issue cost per VALU instruction (cycles).

bench.py multiplies that mean by the launch's SQ_INSTS_VALU (rocprofv3) to
get the launch's issue floor, and reports the measured launch against it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import re
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASM = os.path.join(ROOT, "ilias_net2_amd", "csrc", "build", "sha2_kernels.s")
PROBE = os.path.join(ROOT, "profiles", "round1", "valu_probe.json")
# explicit-register probe (tools/gen_bank_probe.py): VGPR banks, slow/fast
# sequences and the Sigma-shaped mix
SEQ_PROBE = os.path.join(ROOT, "profiles", "round1", "valu_bank_seq_probe.json")
MIXED_ROW = "mix: 3 rot + bitop3 (Sigma), 3-bank"
OUT = os.path.join(ROOT, "profiles", "isa_mix.json")

# bench config -> mangled-name prefix of the kernel instance it launches
KERNELS = {
    "c2": "_ZN4net23dev12fixed_kernelINS0_7Sha256TILb1ELb1ELb1ELb0EEELi0ELb1E",
    "c4": "_ZN4net23dev12fixed_kernelINS0_6Sha512ELi0ELb1E",
    "c3": "_ZN4net23dev10var_kernelINS0_7Sha256TILb1ELb1ELb1ELb0EEE",
    # HMAC instances: <H, PADCONST, MODE, IS384>
    "hmac": "_ZN4net23dev11hmac_kernelINS0_7Sha256TILb1ELb1ELb1ELb0EEELb1ELi0ELb0E",
    "hmac_mtu": "_ZN4net23dev11hmac_kernelINS0_7Sha256TILb1ELb1ELb1ELb0EEELb0ELi0ELb0E",
    "hmac512": "_ZN4net23dev11hmac_kernelINS0_8Sha512HFELb1ELi0ELb0E",
    "hmac512_mtu": "_ZN4net23dev11hmac_kernelINS0_7Sha512HELb0ELi0ELb0E",
    "c3_512": "_ZN4net23dev10var_kernelINS0_7Sha512VE",
    "hmac_verify_mtu": "_ZN4net23dev11hmac_kernelINS0_7Sha256TILb1ELb1ELb1ELb0EEELb0ELi2ELb0E",
    "hmac512_verify_mtu": "_ZN4net23dev11hmac_kernelINS0_7Sha512HELb0ELi2ELb0E",
    "burst_rx": "_ZN4net23dev11hmac_kernelINS0_7Sha512HELb0ELi3ELb0E",
    "burst_tx": "_ZN4net23dev11hmac_kernelINS0_7Sha512HELb0ELi4ELb0E",
    "burst_rx256": "_ZN4net23dev11hmac_kernelINS0_7Sha256TILb1ELb1ELb1ELb0EEELb0ELi3ELb0E",
}

# probe row name -> (mnemonic, operand form); form "v" = VGPR/inline-constant
# sources only, "s" = an SGPR source, "lit" = a 32-bit literal.
PROBE_ROWS = {
    "v_add_u32 (VOP2, v,v)": ("v_add_u32", "v"),
    "v_add_u32 literal": ("v_add_u32", "lit"),
    "v_add_u32 s": ("v_add_u32", "s"),
    "v_xor_b32 (VOP2)": ("v_xor_b32", "v"),
    "v_or_b32 (VOP2)": ("v_or_b32", "v"),
    "v_and_b32": ("v_and_b32", "v"),
    "v_not_b32": ("v_not_b32", "v"),
    "v_sub_u32": ("v_sub_u32", "v"),
    "v_mov_b32": ("v_mov_b32", "v"),
    "v_lshrrev_b32 (VOP2, imm)": ("v_lshrrev_b32", "v"),
    "v_lshlrev_b32 (VOP2, imm)": ("v_lshlrev_b32", "v"),
    "v_bitop3_b32 xor3 (3 v)": ("v_bitop3_b32", "v"),
    "v_alignbit_b32 x,x,imm (rotate)": ("v_alignbit_b32", "v"),
    "v_alignbit_b32 x,x,s": ("v_alignbit_b32", "s"),
    "v_alignbyte_b32 imm": ("v_alignbyte_b32", "v"),
    "v_add3_u32 v,v,v": ("v_add3_u32", "v"),
    "v_add3_u32 v,v,s": ("v_add3_u32", "s"),
    "v_perm_b32 0,v,s (bswap)": ("v_perm_b32", "s"),
    "v_bfi_b32": ("v_bfi_b32", "v"),
    "v_lshl_or_b32 v,imm,v": ("v_lshl_or_b32", "v"),
    "v_and_or_b32": ("v_and_or_b32", "v"),
    "v_or3_b32": ("v_or3_b32", "v"),
    "v_xad_u32": ("v_xad_u32", "v"),
    "v_lshl_add_u64 v,0,v (64-bit add)": ("v_lshl_add_u64", "v"),
    "v_lshl_add_u64 v,0,s": ("v_lshl_add_u64", "s"),
    "v_lshrrev_b64 imm": ("v_lshrrev_b64", "v"),
    "v_add_f32": ("v_add_f32", "v"),
}
# Instructions whose VGPR/SGPR forms measured the same (cost of either row).
SAME_FORMS = {"v_alignbit_b32", "v_add3_u32", "v_perm_b32", "v_lshl_add_u64"}


def cost_table(probe_path=PROBE):
    with open(probe_path) as f:
        rows = json.load(f)["results"]
    t = {}
    for r in rows:
        if r["waves_per_simd"] != 8 or r["op"] not in PROBE_ROWS:
            continue
        t[PROBE_ROWS[r["op"]]] = r["simd_cycles_per_wave_instr_at_2.4GHz"]
    # bitop3: the explicit-register rows of the bank probe (2.5-2.6; the
    # first probe's 3.6-3.8 came from its operand placement, not the op)
    with open(SEQ_PROBE) as f:
        seq = json.load(f)["results"]
    b3 = [r["simd_cycles_per_wave_instr_at_2.4GHz"] for r in seq
          if r["op"].startswith("v_bitop3_b32")]
    t[("v_bitop3_b32", "v")] = sum(b3) / len(b3)
    return t


def kernel_body(lines, prefix):
    start = next(i for i, ln in enumerate(lines)
                 if ln.startswith(prefix) and re.match(r"^\S+:(\s|$)", ln))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    return lines[start:end + 1]


def innermost_loop(body):
    """Lines of the innermost (deepest) loop: every basic block LLVM
    annotates as belonging to it (`in Loop: Header=BBx_y`) plus the header
    block itself, wherever the layout put them (rotated loops place the body
    before the header)."""
    blocks = []             # (label line index, annotation) per basic block
    for i, ln in enumerate(body):
        if re.match(r"^\.LBB\d+_\d+:", ln):
            blocks.append(i)
    blocks.append(len(body))
    best = None
    for i, ln in enumerate(body):
        m = re.match(r"^\.LBB(\d+_\d+):.*Loop Header: Depth=(\d+)", ln)
        if not m:
            continue
        tag, depth = m.group(1), int(m.group(2))
        lines = []
        for b0, b1 in zip(blocks, blocks[1:]):
            head = body[b0]
            if head.startswith(".LBB" + tag + ":") or (
                    "Header=BB" + tag + " " in head + " "):
                lines.extend(body[b0:b1])
        n_valu = sum(1 for l2 in lines if l2.strip().startswith("v_"))
        key = (depth, n_valu)
        if best is None or key > best[0]:
            best = (key, lines)
    return best[1] if best else []


def classify(line):
    parts = line.strip().split(None, 1)
    mn = re.sub(r"_e(32|64)$", "", parts[0])
    ops = parts[1].split(",")[1:] if len(parts) > 1 else []
    form = "v"
    for o in ops:
        o = o.strip().split()[0] if o.strip() else ""
        if re.match(r"^s(\d+|\[)", o):
            form = "s"
        elif re.match(r"^0x[0-9a-f]+$", o) and int(o, 16) > 64:
            form = "lit" if form == "v" else form
    return mn, form


def price(mn, form, table):
    if (mn, form) in table:
        return table[(mn, form)], "measured"
    if mn in SAME_FORMS:
        for f in ("v", "s"):
            if (mn, f) in table:
                return table[(mn, f)], "measured (other operand form)"
    if (mn, "v") in table and form == "lit":
        return table[(mn, "v")], "measured (VGPR form)"
    if (mn, "v") in table and form == "s":
        # an SGPR source moved every fast VOP2 probe to the slow class
        return max(table[(mn, "v")], table[("v_add_u32", "s")]), "VOP2+SGPR class"
    return 4.3, "unprobed: slow-class cost assumed"


def mixed_stream_cost(path=SEQ_PROBE):
    """Issue cost per instruction of a stream that mixes half-rate
    (v_alignbit, v_add3, ...) and full-rate (v_bitop3, v_add, ...) ops.

    The sequence rows of the bank probe show that in such a stream every
    instruction issues at ~4 cycles whatever its class (S F S F: 4.11,
    S F F F: 4.09, 8 S then 8 F: 3.87), so the binding floor is the
    instruction count times the cost of the round-shaped mix (three
    rotates + one bitop3, 3.95)."""
    with open(path) as f:
        rows = json.load(f)["results"]
    return next(r["simd_cycles_per_wave_instr_at_2.4GHz"] for r in rows
                if r["op"] == MIXED_ROW)


def analyse(lines, prefix, table):
    body = kernel_body(lines, prefix)
    loop = innermost_loop(body)
    mix = Counter()
    for ln in loop:
        s = ln.strip()
        if s.startswith("v_"):
            mix[classify(s)] += 1
    total_instr = sum(mix.values())
    cyc = 0.0
    rows = []
    for (mn, form), n in sorted(mix.items(), key=lambda kv: -kv[1]):
        c, how = price(mn, form, table)
        cyc += c * n
        rows.append({"instr": mn, "operands": form, "count": n,
                     "cycles_each": round(c, 3), "priced": how})
    mixed = mixed_stream_cost()
    kinds = {("fast" if table.get((r["instr"], r["operands"]), 4.3) < 3.0 else "slow")
             for r in rows}
    return {"kernel": prefix, "loop_valu_instr": total_instr,
            # binding model: a mixed stream issues every instruction at the
            # Sigma-shaped mix's cost (mixed_stream_cost)
            "mean_issue_cycles_per_valu_instr": (mixed if kinds == {"fast", "slow"}
                                                 else round(cyc / total_instr, 4)) if total_instr else None,
            "model": "mixed-stream: instructions x %s (%s)" % (mixed, MIXED_ROW),
            # optimistic: each instruction at its own pure-stream cost
            "additive_issue_cycles": round(cyc, 1),
            "additive_mean_cycles_per_valu_instr": round(cyc / total_instr, 4) if total_instr else None,
            "mix": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default=ASM)
    ap.add_argument("--out", default=OUT)
    args = ap.parse_args()
    with open(args.asm) as f:
        lines = f.read().splitlines()
    table = cost_table()
    res = {"source": "tools/isa_mix.py over `make asm` output; costs from "
                     "profiles/round1/valu_probe.json (SIMD cycles per wave64 "
                     "instruction at 2.4 GHz, 8 waves/SIMD)",
           "mixed_stream_source": SEQ_PROBE.replace(ROOT + "/", ""),
           "configs": {}}
    # the kernel build the asm came from (make asm and the library share
    # the sources; bench.py ignores the mix of another build)
    sys.path.insert(0, ROOT)
    from ilias_net2_amd import _lib
    res["kernel_build_id"] = _lib.lib().net2_sha2_build_id().decode()
    for cfg, prefix in KERNELS.items():
        res["configs"][cfg] = analyse(lines, prefix, table)
        r = res["configs"][cfg]
        print(f"{cfg:12s} loop VALU {r['loop_valu_instr']:5d}  mean "
              f"{r['mean_issue_cycles_per_valu_instr']} cyc/instr")
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
