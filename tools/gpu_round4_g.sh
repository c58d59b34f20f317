# Round 4: per-length split of burst RX, and the verify / burst bench lines
# again against the mode-selected PMC summaries.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/gpu_burst_bins.sh > /dev/null 2>&1
rc=$?; echo "burst bins rc=$rc"; cat gpurun_out/burst_bins.txt; [ $rc -ne 0 ] && exit $rc
for c in hmac_verify_mtu hmac512_verify_mtu burst_rx burst_tx; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  tail -1 gpurun_out/bench_$c.log | cut -c1-200
done
