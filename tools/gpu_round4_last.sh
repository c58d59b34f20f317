# Round 4, last build: parity tests, smoke, the rocprofv3 round (trace + PMC
# passes per config, stamped with this build), then the default bench line
# and every config against those summaries.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
rc=$?; [ $rc -ne 0 ] && exit $rc
ROUND=round4 bash tools/gpu_profile_round.sh > gpurun_out/profile_round.log 2>&1
rc=$?; echo "profile rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/profile_round.log; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench default rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
SKIP_PYTEST=1 bash tools/gpu_bench_all.sh
