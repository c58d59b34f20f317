#!/usr/bin/env python3
"""Markdown rows of DESIGN.md §6's per-config table from `bench.py --config`
lines (one file per config, the JSON line last), e.g. the outputs of
tools/gpu_bench_all.sh:

  python tools/bench_table.py profiles/round6/bench_*.json

Columns: G/s, kernel ms of the step, HBM GB/s (fraction of 8 TB/s), traffic
over algorithmic bytes, SIMD cycles per VALU instruction, the dominant
kernel's issue-floor fraction (at the counters' clock and, in brackets, at
the timed clock), and the floor fraction of every launch of the step.  A
line whose counters were refused (other build, clock more than 3 % off) shows
"—" there and its timed clock.
"""
import json
import os
import sys


def row(path):
    with open(path) as f:
        d = json.loads([ln for ln in f if ln.startswith("{")][-1])
    cfg = os.path.basename(path).rsplit(".", 1)[0].replace("bench_", "")
    r = d["roofline"]
    v = d.get("roofline_valu") or {}
    fl = v.get("issue_floor") or {}
    st = fl.get("step") or {}
    sclk = d.get("gpu", {}).get("sclk_mhz_during_timed_steps")
    if r.get("traffic") is None:
        return (f"| {cfg} | {d['value'] / 1e9:.3f} | {r['kernel_ms']:.4f} | "
                f"{r['achieved']:,.0f} ({r['frac']:.3f}) | — (refused, "
                f"timed at {sclk} MHz) | — | — | — |")
    step = (f"{st['frac_at_timed_sclk']:.2f}" if len(st.get("kernels", [])) > 1
            else "= dominant")
    return (f"| {cfg} | {d['value'] / 1e9:.3f} | {r['kernel_ms']:.4f} | "
            f"{r['achieved']:,.0f} ({r['frac']:.3f}) | "
            f"{r['traffic_over_algorithmic']:.3f} | "
            f"{v['simd_cycles_per_valu_instr']:.2f} | "
            f"{fl['frac']:.2f} ({fl['frac_at_timed_sclk']:.2f}) | {step} |")


if __name__ == "__main__":
    print("| config | G/s | kernel ms | HBM GB/s (frac of 8 TB/s) | traffic / "
          "algorithmic | SIMD cycles per VALU instr | issue-floor frac ±0.02 "
          "(at the timed clock) | step floor frac ±0.02 |")
    print("|---|---|---|---|---|---|---|---|")
    for p in sys.argv[1:]:
        print(row(p))
