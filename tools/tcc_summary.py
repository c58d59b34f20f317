#!/usr/bin/env python3
"""Summarise tools/gpu_tcc_calib.sh: per-launch L2 (TCC) read requests of the
config's dominant kernel by size, and the bytes they stand for.

TCC_EA0_RDREQ counts every read request the L2 sends to memory,
TCC_EA0_RDREQ_32B / _64B the 32- and 64-byte ones; the rest are 128-byte
requests.  C2 (1 GiB read exactly once, 16 B/lane) calibrates the reading:
its request bytes must come out at the payload.  Writes
profiles/<round>/tcc_<cfg>.json.
"""
import argparse
import csv
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = {"c2": "fixed_kernel<net2::dev::Sha256", "c4": "fixed_kernel<net2::dev::Sha512",
          "c3": "var_kernel<net2::dev::Sha256", "c3_512": "var_kernel<net2::dev::Sha512",
          "hmac512_verify_mtu": "hmac_kernel<net2::dev::Sha512",
          "burst_rx": "hmac_kernel<net2::dev::Sha512", "burst_tx": "hmac_kernel<net2::dev::Sha512"}
ALGO = {"c2": 1 << 30, "c4": 1 << 30, "c3": None}


def per_dispatch(path, pat):
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if pat not in r["Kernel_Name"]:
                continue
            k = (r["Dispatch_Id"], r["Counter_Name"])
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    out = {}
    for (d, c), v in vals.items():
        out.setdefault(c, []).append(v)
    return {c: statistics.median(v) for c, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", required=True)
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--round", default="round2")
    ap.add_argument("--payload", type=float, default=None,
                    help="algorithmic read bytes per launch (default: C2/C4 1 GiB)")
    a = ap.parse_args()
    med = {}
    for tag in ("TCC_EA0_RDREQ", "TCC_EA0_RDREQ_DRAM"):
        p = os.path.join(a.src, f"tcc_{a.cfg}_{tag}", "run_counter_collection.csv")
        if os.path.exists(p):
            med.update(per_dispatch(p, KERNEL[a.cfg]))
    r = med.get("TCC_EA0_RDREQ", 0)
    r32 = med.get("TCC_EA0_RDREQ_32B", 0)
    r64 = med.get("TCC_EA0_RDREQ_64B", 0)
    r128 = r - r32 - r64
    byts = 128 * r128 + 64 * r64 + 32 * r32
    res = {"config": a.cfg, "kernel": KERNEL[a.cfg], "counters_median_per_launch": med,
           "requests": {"128B": r128, "64B": r64, "32B": r32},
           "read_bytes_from_requests": byts}
    algo = a.payload or ALGO.get(a.cfg)
    if algo:
        res["algorithmic_read_bytes"] = algo
        res["ratio"] = byts / algo
    dst = os.path.join(ROOT, "profiles", a.round)
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, f"tcc_{a.cfg}.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
