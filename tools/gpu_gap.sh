set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/kernel_ab > gpurun_out/kernel_ab2.json 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 50 --warmup 20 --no-cpu-baseline > gpurun_out/bench_long.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_short.log 2>&1 || exit $?
timeout -k 10 120 ./tools/kernel_ab > gpurun_out/kernel_ab3.json 2>&1 || exit $?
