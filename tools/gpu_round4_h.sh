# Round 4: 8,192-packet binning tiles (128 workgroups per 1 M) against the
# shipped 4,096 -- stamps and library A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in probe probe32; do
  NET2_SHA2_LIB=$PWD/tools/ab/$v.so timeout -k 10 200 python tools/bin_probe.py > gpurun_out/bin_probe_$v.txt 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -v -e Warn -e amdgpu.ids gpurun_out/bin_probe_$v.txt; [ $rc -ne 0 ] && exit $rc
done
NET2_SHA2_LIB=$PWD/tools/ab/items32.so timeout -k 10 300 python -u -m pytest tests/test_gpu_binning.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_items32.log 2>&1
rc=$?; echo "pytest items32 rc=$rc"; tail -2 gpurun_out/gputest_items32.log; [ $rc -ne 0 ] && exit $rc
rm -f tools/ab/probe*.so
CFGS=${CFGS:-"c3 c3_512 hmac512_verify_mtu burst_rx"} REPS=${REPS:-"1 2"} bash tools/gpu_ab_lib.sh > /dev/null
cat gpurun_out/ab_lib.txt
