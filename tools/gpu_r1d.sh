# GPU parity suite for the current build, then the VGPR-bank probe.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./tools/bank_probe > gpurun_out/bank_probe.json
rc=$?; echo "bank rc=$rc"; cat gpurun_out/bank_probe.json; exit $rc
