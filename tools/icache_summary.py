#!/usr/bin/env python3
"""Median per launch of the instruction-cache counters tools/gpu_icache.sh
collected, for each config's kernel (tools/pmc_summary.py's KERNEL map)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import KERNEL, per_dispatch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = {}
for cfg in sys.argv[1:]:
    med = {}
    for tag in ("SQC_ICACHE_HITS", "SQ_IFETCH"):
        path = os.path.join(ROOT, "gpurun_out", f"ic_{cfg}_{tag}", "run_counter_collection.csv")
        if os.path.exists(path):
            c, _ = per_dispatch(path, KERNEL[cfg])
            med.update({k: statistics.median(v) for k, v in c.items()})
    h, m = med.get("SQC_ICACHE_HITS"), med.get("SQC_ICACHE_MISSES")
    if h is not None and m is not None and h + m > 0:
        med["icache_miss_rate"] = m / (h + m)
    out[cfg] = med
print(json.dumps(out, indent=1, sort_keys=True))
