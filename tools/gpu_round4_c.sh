# Round 4: parity of the short-tail build, kernel traces of C3 / burst RX
# (binning launch durations), the library A/B (one address path, one-pass
# binning, short tail two per lane), then the default bench line.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
NET2_SHA2_LIB=$PWD/tools/ab/short2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_packet.py tests/test_gpu_dgram.py tests/test_gpu_binning.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_short2.log 2>&1
rc=$?; echo "pytest short2 rc=$rc"; tail -2 gpurun_out/gputest_short2.log; [ $rc -ne 0 ] && exit $rc
for c in c3 burst_rx; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --no-extras --steps 20 > gpurun_out/prof_$c.log 2>&1
  rc=$?; echo "trace $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  f=$(find gpurun_out/prof_$c -name "*kernel_stats.csv" | head -1); cut -c1-160 $f | head -8
done
CFGS=${CFGS:-"c3 c3_512 hmac_verify_mtu hmac512_mtu hmac512_verify_mtu burst_rx burst_tx"} REPS=${REPS:-"1 2"} bash tools/gpu_ab_lib.sh
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench default rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-400
