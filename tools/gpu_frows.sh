# Measurements for the SURVEY 8f rows: HMAC, ph_to_iv, signed-payload flow.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in hmac hmac_mtu ph_iv; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  tail -1 gpurun_out/bench_$c.log
done
timeout -k 10 600 python tools/bench_sign.py > gpurun_out/bench_sign.log 2>&1
rc=$?; echo "bench_sign rc=$rc"; cat gpurun_out/bench_sign.log; [ $rc -ne 0 ] && exit $rc
CFGS="hmac hmac_mtu" bash tools/gpu_profile.sh > gpurun_out/prof_frows.log 2>&1
echo "profile rc=$?"
exit 0
