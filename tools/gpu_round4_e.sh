# Round 4: one-pass binning barrier ordering -- per-phase stamps for the
# three fence levels, the binning tests on the relaxed build, kernel traces
# and an A/B against the three-launch binning.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in probe probe0 probe2; do
  NET2_SHA2_LIB=$PWD/tools/ab/$v.so timeout -k 10 200 python tools/bin_probe.py > gpurun_out/bin_probe_$v.txt 2>&1
  rc=$?; echo "== $v rc=$rc"; cat gpurun_out/bin_probe_$v.txt | grep -v Warn; [ $rc -ne 0 ] && exit $rc
done
NET2_SHA2_LIB=$PWD/tools/ab/fence0.so timeout -k 10 300 python -u -m pytest tests/test_gpu_binning.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_fence0.log 2>&1
rc=$?; echo "pytest fence0 rc=$rc"; tail -2 gpurun_out/gputest_fence0.log; [ $rc -ne 0 ] && exit $rc
for v in default fence0; do
  if [ $v = default ]; then unset NET2_SHA2_LIB; else export NET2_SHA2_LIB=$PWD/tools/ab/$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${v}_c3 -o run --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline --no-extras --steps 20 > gpurun_out/prof_${v}_c3.log 2>&1
  rc=$?; echo "trace $v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  grep -E "bin_" gpurun_out/prof_${v}_c3/run_kernel_stats.csv | cut -d, -f1-7 | sed 's/(.*)"/"/'
done
unset NET2_SHA2_LIB
rm -f tools/ab/probe*.so
CFGS=${CFGS:-"c3 c3_512 burst_rx"} REPS=${REPS:-"1 2"} bash tools/gpu_ab_lib.sh > /dev/null
cat gpurun_out/ab_lib.txt
