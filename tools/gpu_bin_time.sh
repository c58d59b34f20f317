# Binned-path parity and per-kernel times of the binning launches for the
# in-tree library and each tools/ab/*.so (C3 shape).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in default tools/ab/*.so; do
  if [ "$lib" = default ]; then unset NET2_SHA2_LIB; tag=default; else export NET2_SHA2_LIB=$PWD/$lib; tag=$(basename $lib .so); fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "var or config3 or hmac" > gpurun_out/pytest_bin.log 2>&1
  rc=$?; echo "parity $tag rc=$rc"; tail -1 gpurun_out/pytest_bin.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/bt_$tag -o run --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline --no-extras --steps 20 > gpurun_out/bt_$tag.log 2>&1
  rc=$?; echo "trace $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 -c "
import csv,glob
f=glob.glob('gpurun_out/bt_$tag/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'bin_' in r['Name'] or 'var_kernel' in r['Name'] or 'fill' in r['Name']: print('$tag', r['Name'][:40], r['AverageNs'])"
done
