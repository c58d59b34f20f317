#!/usr/bin/env python3
"""The driver's bench command under rocprofv3 --kernel-trace --stats: the
dominant kernels' trace averages next to the line's own HIP-event kernel
times (tools/gpu_round_final.sh STAGE=trace_default).
  default_trace_summary.py KERNEL_STATS_CSV BENCH_LOG [KERNEL_TRACE_CSV]
With the per-dispatch trace, each kernel is also averaged over its launches
of 1 M work-items only (the line's 1 M-packet steps; the e2e chunks and
C1's small batches run the same kernels on fewer packets)."""
import csv
import json
import sys

# kernel-name fragments of the line's configs: headline C2, C3, C4
PICK = {"c2": ("fixed_kernel<net2::dev::Sha256", "Li0ELb1E", "0, true>"),
        "c4": ("fixed_kernel<net2::dev::Sha512", "", "0, true>"),
        "c3": ("var_kernel<net2::dev::Sha256", "", ""),
        "c3_binning": ("bin_onepass_kernel", "", "")}


def main():
    stats = list(csv.DictReader(open(sys.argv[1])))
    line = None
    for ln in open(sys.argv[2]):
        if ln.startswith("{"):
            line = json.loads(ln)
    out = {"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 "
                      "--steps 20 --warmup 5 (the driver's N=1 command)",
           "line_value_digests_per_s": line and line["value"],
           "line_kernel_ms_hip_events": line and line["roofline"]["kernel_ms"],
           "line_extra_kernel_ms": line and {k: (v.get("roofline") or {}).get("kernel_ms")
                                             for k, v in line.get("extra_configs", {}).items()
                                             if k in ("c3", "c4")},
           "line_gpu": line and line.get("gpu"),
           "kernel_stats": "kernel_stats_default_cmd.csv (every launch of the run: "
                           "warmups, the e2e and burst e2e chunks, C1's small batches)"}
    trace = list(csv.DictReader(open(sys.argv[3]))) if len(sys.argv) > 3 else []
    for key, (frag, _, tail) in PICK.items():
        rows = [r for r in stats if frag in r["Name"] and (not tail or tail in r["Name"])]
        if rows:
            r = max(rows, key=lambda r: int(r["Calls"]))
            out["trace_" + key] = {"name": r["Name"][:90], "launches": int(r["Calls"]),
                                   "avg_us": round(float(r["AverageNs"]) / 1e3, 2)}
            full = [int(d["End_Timestamp"]) - int(d["Start_Timestamp"]) for d in trace
                    if d.get("Kernel_Name") == r["Name"] and
                    int(d.get("Grid_Size") or d.get("Grid_Size_X") or 0) >= (1 << 20)]
            if full:
                out["trace_" + key]["launches_1M"] = len(full)
                out["trace_" + key]["avg_us_1M"] = round(sum(full) / len(full) / 1e3, 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
