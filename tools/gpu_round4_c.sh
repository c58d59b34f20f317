# Round 4: kernel trace of C3 (binning launch durations), then the library
# A/B of the one-path loads and the three-launch binning.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c3 burst_rx; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --no-extras --steps 20 > gpurun_out/prof_$c.log 2>&1
  rc=$?; echo "trace $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  f=$(find gpurun_out/prof_$c -name "*kernel_stats.csv" | head -1); cut -c1-160 $f | head -12
done
CFGS=${CFGS:-"c3 c3_512 hmac_mtu hmac_verify_mtu hmac512_mtu hmac512_verify_mtu burst_rx burst_tx"} REPS=${REPS:-"1 2"} bash tools/gpu_ab_lib.sh
