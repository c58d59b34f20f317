set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in burst_rx burst_tx; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; tail -3 gpurun_out/bench_$c.log; [ $rc -ne 0 ] && exit $rc
done
CFGS="burst_rx burst_tx" bash tools/gpu_profile.sh || exit 1
for c in burst_rx burst_tx; do python3 tools/pmc_summary.py --cfg $c --round round2 > /dev/null || exit 1; cp profiles/pmc_$c.json gpurun_out/; cp profiles/round2/kernel_stats_$c.csv gpurun_out/ ; done
timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_c2_quick.log 2>&1
echo "c2 rc=$?"; tail -1 gpurun_out/bench_c2_quick.log
