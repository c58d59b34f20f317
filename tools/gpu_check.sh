# Parity tests + bench (c2, c4, c3) + kernel trace for each config.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for c in c2 c4 c3; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  tail -1 gpurun_out/bench_$c.log
done
timeout -k 10 300 python bench.py --config c3 --unbinned --no-cpu-baseline > gpurun_out/bench_c3_unbinned.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c3_unbinned.log
for c in c2 c4 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python bench.py --config $c --no-cpu-baseline --steps 20 > gpurun_out/prof_$c.log 2>&1
  rc=$?; echo "rocprof $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
