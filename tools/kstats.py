#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv compactly: kernel (short name), calls,
average / min / max microseconds.  Usage: kstats.py CSV [substring ...]"""
import csv
import sys

keys = sys.argv[2:]
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if keys and not any(k in n for k in keys):
        continue
    short = n.split("(")[0][-56:]
    print(f"{short:56s} calls={r['Calls']:>5} avg={float(r['AverageNs']) / 1e3:8.2f}us "
          f"min={float(r['MinNs']) / 1e3:7.2f} max={float(r['MaxNs']) / 1e3:7.2f}")
