#!/bin/bash
# Per-kernel split of the burst RX step by datagram length
# (tools/burst_bins.py under rocprofv3 --kernel-trace --stats, one process
# per length set) -> gpurun_out/burst_bins/<set>/..._kernel_stats.csv and a
# summary in gpurun_out/burst_bins.txt.
set -eu
export TMPDIR=/tmp
OUT=gpurun_out/burst_bins
mkdir -p $OUT
: > gpurun_out/burst_bins.txt
for set in 136 584 1500 136,584,1500; do
  tag=$(echo $set | tr , _)
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o run --output-format csv -- \
      python3 tools/burst_bins.py --lens $set >> gpurun_out/burst_bins.txt
  f=$(find $OUT/$tag -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$set" >> gpurun_out/burst_bins.txt <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    nm = r["Name"]
    if any(k in nm for k in ("hmac_kernel", "burst_final", "bin_count", "bin_scatter", "bin_onepass", "fillBuffer")):
        print(f"  {sys.argv[2]:14s} {nm.split('(')[0][-60:]:60s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:8.2f}")
EOF
done
cat gpurun_out/burst_bins.txt
