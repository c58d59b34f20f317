# Round 4: where the one-pass binning launch spends its time.  Kernel
# traces of C3 with the shipped library, the acquiring-poll build and the
# three-launch binning, the binning tests, then an A/B against bin3.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_binning.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_binning.log 2>&1
rc=$?; echo "pytest binning rc=$rc"; tail -2 gpurun_out/gputest_binning.log; [ $rc -ne 0 ] && exit $rc
for v in default spinacq bin3; do
  if [ $v = default ]; then unset NET2_SHA2_LIB; else export NET2_SHA2_LIB=$PWD/tools/ab/$v.so; fi
  for c in c3 burst_rx; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${v}_$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --no-extras --steps 20 > gpurun_out/prof_${v}_$c.log 2>&1
    rc=$?; echo "trace $v $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
    f=$(find gpurun_out/prof_${v}_$c -name "*kernel_stats.csv" | head -1); grep -E "bin_|var_kernel|hmac_kernel" $f | cut -d, -f1-5 | sed 's/(.*)"/"/' | cut -c1-150
  done
done
unset NET2_SHA2_LIB
CFGS=${CFGS:-"c3 c3_512 hmac512_verify_mtu burst_rx"} REPS=${REPS:-"1 2"} bash tools/gpu_ab_lib.sh > /dev/null
cat gpurun_out/ab_lib.txt
