set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import torch; print(torch.__version__, torch.cuda.is_available())" > gpurun_out/env.log 2>&1
rocm-smi --showproductname >> gpurun_out/env.log 2>&1 || true
nproc >> gpurun_out/env.log; lscpu | head -20 >> gpurun_out/env.log
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_c2.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cat gpurun_out/bench_c2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1
echo "rocprof rc=$?"
