# Round-1 follow-up: parity suite, benches of every config, c3/hmac512
# kernel traces, SHA-512 constant-read / fence A/B, LDS-staged SHA-256 A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for c in c2 c3 c4; do
timeout -k 10 400 python bench.py --config $c > gpurun_out/bench_$c.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$c.log
done
for c in hmac hmac_mtu hmac512 hmac512_mtu; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value']/1e9, d['ms_per_step'])"
done
for c in c3 hmac512_mtu; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --steps 20 > gpurun_out/prof_$c.log 2>&1 || exit $?
done
for b in kernel_ab kernel_ab_km2 kernel_ab_nofence; do
AB512=1 timeout -k 10 200 ./tools/$b > gpurun_out/ab512_$b.json 2>&1 || exit $?
done
timeout -k 10 200 ./tools/kernel_ab > gpurun_out/ab256.json 2>&1 || exit $?
cat gpurun_out/ab256.json
grep -H S0 gpurun_out/ab512_*.json
exit 0
