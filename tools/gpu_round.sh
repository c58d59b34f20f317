# Parity tests, then the e2e (PCIe-inclusive) bench and an HMAC batch timing.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config e2e --steps 10 --warmup 3 > gpurun_out/bench_e2e.log 2>&1
rc=$?; echo "e2e rc=$rc"; tail -1 gpurun_out/bench_e2e.log; [ $rc -ne 0 ] && exit $rc
exit 0
