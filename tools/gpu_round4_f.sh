# Round 4: one-pass binning with the two-level barrier and capped wave
# aggregation -- tests, per-phase stamps, kernel traces, A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_binning.py tests/test_gpu_parity.py tests/test_gpu_packet.py tests/test_gpu_dgram.py tests/test_gpu_multidev.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_bin2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gputest_bin2.log; [ $rc -ne 0 ] && exit $rc
for v in probe probes1; do
  NET2_SHA2_LIB=$PWD/tools/ab/$v.so timeout -k 10 200 python tools/bin_probe.py > gpurun_out/bin_probe_$v.txt 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -v -e Warn -e amdgpu.ids gpurun_out/bin_probe_$v.txt; [ $rc -ne 0 ] && exit $rc
done
for v in default bin3; do
  if [ $v = default ]; then unset NET2_SHA2_LIB; else export NET2_SHA2_LIB=$PWD/tools/ab/$v.so; fi
  for c in c3 burst_rx; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${v}_$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --no-extras --steps 20 > gpurun_out/prof_${v}_$c.log 2>&1
    rc=$?; echo "trace $v $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python3 tools/kstats.py gpurun_out/prof_${v}_$c/run_kernel_stats.csv bin_ var_kernel hmac_kernel burst_final
  done
done
unset NET2_SHA2_LIB
rm -f tools/ab/probe*.so
CFGS=${CFGS:-"c3 c3_512 hmac_mtu hmac_verify_mtu hmac512_verify_mtu burst_rx"} REPS=${REPS:-"1 2"} bash tools/gpu_ab_lib.sh > /dev/null
cat gpurun_out/ab_lib.txt
