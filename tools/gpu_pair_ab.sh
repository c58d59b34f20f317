# Pair-load A/B: parity per library build, timing through bench.py, and one
# FETCH_SIZE pass per (build, config) to see the HBM re-fetch change.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in default tools/ab/*.so; do
  if [ "$lib" = default ]; then unset NET2_SHA2_LIB; tag=default; else export NET2_SHA2_LIB=$PWD/$lib; tag=$(basename $lib .so); fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fixed or var or config or hmac" > gpurun_out/pytest_pair.log 2>&1
  rc=$?; echo "parity $tag rc=$rc"; tail -1 gpurun_out/pytest_pair.log; [ $rc -ne 0 ] && exit $rc
  for c in ${PMC_CFGS:-c2 c3}; do
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fpair_${tag}_$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --prewarm-ms 100 --no-cpu-baseline --no-extras > gpurun_out/fpair_${tag}_$c.log 2>&1
    rc=$?; echo "pmc $tag $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
unset NET2_SHA2_LIB
CFGS=${AB_CFGS:-"c2 c3 hmac hmac_mtu"} bash tools/gpu_ab_lib.sh
