# Parity tests, then every bench config (device-resident + e2e); one JSON
# line per config under gpurun_out/bench_<cfg>.log.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_PYTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
for c in ${CFGS:-c2 c4 c3 c3_512 hmac hmac_mtu hmac_verify_mtu hmac512 hmac512_mtu hmac512_verify_mtu burst_rx burst_tx burst_rx256 ph_iv e2e}; do
  extra=""
  [ "$c" = e2e ] && extra="--steps 10 --warmup 3"
  timeout -k 10 300 python bench.py --config $c $extra > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  tail -1 gpurun_out/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value']/1e9,4), 'G/s', d['ms_per_step'], 'ms', d.get('roofline',{}).get('kernel_ms'))"
done
exit 0
