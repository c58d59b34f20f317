#!/usr/bin/env python3
"""Fold tools/c3_traffic.py runs into profiles/<round>/c3_traffic_layouts.json:
a `rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B` pass
(gpurun_out/c3t_pmc) and a `--kernel-trace` pass (gpurun_out/c3t_trace).
var_kernel dispatches come 5 per layout, in the script's order."""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth  # noqa: E402

LAYOUTS = ["packed back to back (BASELINE C3)",
           "every start rounded up to 16 bytes (net2_sha2_batch's packer)",
           "every start rounded up to 128 bytes (no shared lines, line-aligned block pairs)",
           "packed, unbinned (memory order)"]


def main(rnd="round2"):
    src = os.path.join(ROOT, "gpurun_out")
    req = {}
    with open(os.path.join(src, "c3t_pmc", "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if "var_kernel" not in r["Kernel_Name"]:
                continue
            k = (int(r["Dispatch_Id"]), r["Counter_Name"])
            req[k] = req.get(k, 0.0) + float(r["Counter_Value"])
    ids = sorted({d for d, _ in req})
    dur = []
    with open(os.path.join(src, "c3t_trace", "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            if "var_kernel" in r["Kernel_Name"]:
                dur.append((int(r["Start_Timestamp"]),
                            int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    dur = [d for _, d in sorted(dur)]
    lens = synth.mixed_lengths(3, 1 << 20)
    payload = int(lens.sum())
    algo = payload + (1 << 20) * (32 + 12)
    out = {"what": "C3 batch (1 M x {64, 512, 1500} B, seeds 3/4) hashed by var_kernel from four "
                   "layouts, tools/c3_traffic.py under rocprofv3 --pmc TCC_EA0_RDREQ "
                   "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B and --kernel-trace (5 launches per "
                   "layout, medians); folded by tools/c3_traffic_summary.py",
           "payload_bytes": payload, "algorithmic_bytes_per_launch": algo, "layouts": {},
           "var_kernel_us_under_tracing": {}}
    for li, name in enumerate(LAYOUTS):
        sel = ids[5 * li:5 * li + 5]
        r = statistics.median(req.get((d, "TCC_EA0_RDREQ"), 0) for d in sel)
        r32 = statistics.median(req.get((d, "TCC_EA0_RDREQ_32B"), 0) for d in sel)
        r64 = statistics.median(req.get((d, "TCC_EA0_RDREQ_64B"), 0) for d in sel)
        rb = 128 * (r - r32 - r64) + 64 * r64 + 32 * r32
        row = {"read_requests": r, "read_bytes": rb,
               "read_plus_digest_write_over_algorithmic": round((rb + (1 << 20) * 32) / algo, 3)}
        out["layouts"][name] = row
        if dur:
            out["var_kernel_us_under_tracing"][name] = round(
                statistics.median(dur[5 * li:5 * li + 5]) / 1e3, 1)
    dst = os.path.join(ROOT, "profiles", rnd, "c3_traffic_layouts.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
