set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
for c in c3 hmac_mtu; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value']/1e9, d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline --steps 20 > gpurun_out/prof_c3.log 2>&1 || exit $?

AB512=1 timeout -k 10 200 ./tools/kernel_ab > gpurun_out/ab512_base.json 2>&1 || exit $?
AB512=1 timeout -k 10 200 ./tools/kernel_ab_shr > gpurun_out/ab512_shr.json 2>&1 || exit $?
AB512=1 timeout -k 10 200 ./tools/kernel_ab > gpurun_out/ab512_base2.json 2>&1 || exit $?
timeout -k 10 200 ./tools/kernel_ab > gpurun_out/ab256.json 2>&1 || exit $?
cat gpurun_out/ab256.json
grep S0 gpurun_out/ab512_base.json gpurun_out/ab512_shr.json gpurun_out/ab512_base2.json
exit 0
