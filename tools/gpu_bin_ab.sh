# Binning variants: parity of the binned paths per library build, then the
# in-process-shape A/B of bench configs that bin (tools/gpu_ab_lib.sh).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in default tools/ab/*.so; do
  if [ "$lib" = default ]; then unset NET2_SHA2_LIB; else export NET2_SHA2_LIB_ALLOW_OLD_ABI=1 NET2_SHA2_LIB=$PWD/$lib; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "var or config3 or hmac" > gpurun_out/pytest_bin.log 2>&1
  rc=$?; echo "parity $lib rc=$rc"; tail -1 gpurun_out/pytest_bin.log; [ $rc -ne 0 ] && exit $rc
done
unset NET2_SHA2_LIB
CFGS="c3 hmac_mtu" bash tools/gpu_ab_lib.sh
