#!/usr/bin/env python3
"""Fold rocprofv3 outputs into the per-launch numbers bench.py reports.

Inputs (produced by tools/gpu_profile.sh on the GPU box, one rocprofv3 call
per counter group -- PMC passes are never combined with tracing):
  gpurun_out/prof_<cfg>/run_kernel_stats.csv            --kernel-trace --stats
  gpurun_out/pmc_<cfg>_<group>/run_counter_collection.csv   --pmc <group>

Output: profiles/pmc_<cfg>.json and a copy of the kernel-stats CSV under
profiles/<round>/.

Corrections (MI355X_MICROARCH.md, "HBM" and "rocprofv3 PMC slots"):
  * FETCH_SIZE / WRITE_SIZE are in KiB; x1024 for bytes.
  * gfx950 FETCH_SIZE counts exactly half the bytes of a 16 B/lane read
    stream (128-B requests tallied as 64 B): our block loads are
    global_load_dwordx4 (16 B/lane), so FETCH_SIZE is doubled.
  * WRITE_SIZE is exact for 16 B/lane stores (digests are dwordx4 stores).
  * GRBM_GUI_ACTIVE is summed over the 8 XCDs: clock = value / 8 / duration.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = {"c2": "fixed_kernel<net2::dev::Sha256", "c4": "fixed_kernel<net2::dev::Sha512",
          "c3": "var_kernel<net2::dev::Sha256", "c3_512": "var_kernel<net2::dev::Sha512",
          "hmac": "hmac_kernel<net2::dev::Sha256",
          "hmac_mtu": "hmac_kernel<net2::dev::Sha256", "ph_iv": "ph_iv_kernel",
          "hmac512": "hmac_kernel<net2::dev::Sha512", "hmac512_mtu": "hmac_kernel<net2::dev::Sha512",
          "hmac_verify_mtu": "hmac_kernel<net2::dev::Sha256",
          "hmac512_verify_mtu": "hmac_kernel<net2::dev::Sha512",
          "burst_rx": "hmac_kernel<net2::dev::Sha512", "burst_tx": "hmac_kernel<net2::dev::Sha512",
          "burst_rx256": "hmac_kernel<net2::dev::Sha256"}
# the timed kernel's HMAC mode (the template's last argument), where the
# config also runs another mode once, untimed: the signing pass before a
# verify config, the encode before burst RX
# (hmac_kernel<H, PADCONST, MODE, IS384>: these configs run IS384 = false)
MODE = {"hmac_verify_mtu": ", 2, false>", "hmac512_verify_mtu": ", 2, false>",
        "burst_rx": ", 3, false>", "burst_tx": ", 4, false>", "burst_rx256": ", 3, false>"}


def matches(name, cfg):
    return KERNEL[cfg] in name and MODE.get(cfg, "") in name


def per_dispatch(path, cfg):
    """{counter: [per-dispatch totals]} and [durations ns] for one kernel."""
    vals, durs = {}, {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if not matches(r["Kernel_Name"], cfg):
                continue
            d = r["Dispatch_Id"]
            key = (d, r["Counter_Name"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
            durs[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for (d, c), v in vals.items():
        out.setdefault(c, []).append(v)
    return out, list(durs.values())


def step_kernels(path, cfg, counter="SQ_INSTS_VALU"):
    """The library's kernels that run once per step beside the dominant one
    (binning, the burst final kernel): {short name: (dispatches, median
    counter per dispatch)}, kernels dispatched about as often as the
    dominant one only (not the untimed set-up launches)."""
    vals, names = {}, {}
    with open(path) as f:
        for r in csv.DictReader(f):
            nm = r["Kernel_Name"]
            if "net2::dev::" not in nm or r["Counter_Name"] != counter:
                continue
            d = r["Dispatch_Id"]
            vals[(nm, d)] = vals.get((nm, d), 0.0) + float(r["Counter_Value"])
    for (nm, d), v in vals.items():
        names.setdefault(nm, []).append(v)
    dom = [v for nm, v in names.items() if matches(nm, cfg)]
    if not dom:
        return {}
    ndom = len(dom[0])
    out = {}
    for nm, v in names.items():
        if len(v) >= 0.9 * ndom:
            short = nm.split("(")[0].replace("void ", "").replace("net2::dev::", "")
            out[short] = {"dispatches": len(v), "median_per_dispatch": statistics.median(v),
                          "dominant": matches(nm, cfg)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", required=True, choices=sorted(KERNEL))
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--round", default="round1")
    args = ap.parse_args()
    pat = KERNEL[args.cfg]

    counters, durs_all = {}, []
    tags = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "FETCH_SIZE", "WRITE_SIZE",
            "SQ_INSTS_SALU")
    for tag in tags:
        path = os.path.join(args.src, f"pmc_{args.cfg}_{tag}", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        c, d = per_dispatch(path, args.cfg)
        for k, v in c.items():
            counters[k] = v
        durs_all += d
    med = {k: statistics.median(v) for k, v in counters.items()}
    res = {"config": args.cfg, "kernel": pat + MODE.get(args.cfg, ""), "dispatches_per_pass": len(durs_all) and
           max(len(v) for v in counters.values()),
           "counters_median_per_launch": med}
    # the box and clock the trace pass ran at: its bench.py line (the trace
    # average is only comparable with a bench line of the same clock)
    log = os.path.join(args.src, f"prof_{args.cfg}.log")
    if os.path.exists(log):
        line = None
        with open(log) as f:
            for ln in f:
                if ln.startswith("{"):
                    line = ln
        if line:
            b = json.loads(line)
            g = b.get("gpu", {})
            res["trace_box"] = {"host": g.get("host"), "pci": g.get("pci"),
                                "sclk_mhz_during_timed_steps":
                                    g.get("sclk_mhz_during_timed_steps"),
                                "bench_kernel_ms": b.get("roofline", {}).get("kernel_ms"),
                                "bench_ms_per_step": b.get("ms_per_step")}
    stats_csv = os.path.join(args.src, f"prof_{args.cfg}", "run_kernel_stats.csv")
    if os.path.exists(stats_csv):
        with open(stats_csv) as f:
            for r in csv.DictReader(f):
                if matches(r["Name"], args.cfg):
                    res["trace_avg_ns"] = float(r["AverageNs"])
                    res["trace_calls"] = int(r["Calls"])
        dst = os.path.join(ROOT, "profiles", args.round)
        os.makedirs(dst, exist_ok=True)
        shutil.copy(stats_csv, os.path.join(dst, f"kernel_stats_{args.cfg}.csv"))
    if "FETCH_SIZE" in med:
        fetch = med["FETCH_SIZE"] * 1024 * 2          # KiB -> B, gfx950 x2
        write = med.get("WRITE_SIZE", 0.0) * 1024
        res["hbm_read_bytes_per_launch"] = fetch
        res["hbm_write_bytes_per_launch"] = write
        res["hbm_bytes_per_launch"] = fetch + write
        res["correction"] = "FETCH_SIZE*1024*2 (gfx950 16B/lane half-count) + WRITE_SIZE*1024"
    if "SQ_INSTS_VALU" in med:
        res["valu_wave_instr_per_launch"] = med["SQ_INSTS_VALU"]
        path = os.path.join(args.src, f"pmc_{args.cfg}_SQ_INSTS_VALU", "run_counter_collection.csv")
        sk = step_kernels(path, args.cfg) if os.path.exists(path) else {}
        if sk:
            # every launch of a step: the floor of the whole step, not only
            # of its dominant kernel
            res["step_kernels_valu"] = sk
            res["step_valu_wave_instr"] = sum(k["median_per_dispatch"] for k in sk.values())
    if "GRBM_GUI_ACTIVE" in med and durs_all:
        res["clock_ghz_under_pmc"] = med["GRBM_GUI_ACTIVE"] / 8 / statistics.median(durs_all)
    # the kernel build these counters belong to (bench.py ignores counters
    # of another build); the library the profiled bench.py runs loaded
    sys.path.insert(0, ROOT)
    from ilias_net2_amd import _lib
    res["kernel_build_id"] = _lib.lib().net2_sha2_build_id().decode()
    out = os.path.join(ROOT, "profiles", f"pmc_{args.cfg}.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
