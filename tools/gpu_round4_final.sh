# Round 4 final lines: the default bench line (what the driver runs), then
# every config (tools/gpu_bench_all.sh, parity tests first), all against
# the PMC summaries of the same build.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench default rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_bench_all.sh
