# Round 4: GPU tests, single-payload latency / crossover / long messages,
# then the N>1 gloo rehearsal.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gputest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/latency_long.py > gpurun_out/latency_long.jsonl 2> gpurun_out/latency_long.err
rc=$?; echo "latency rc=$rc"; cat gpurun_out/latency_long.jsonl | cut -c1-300; [ $rc -ne 0 ] && exit $rc

bash tools/gpu_dist.sh
