# A/B of the host path's digest return: kernel stores into pinned host
# memory (default) vs a D2H copy per chunk (NET2_SHA2_D2H_COPY=1).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multidev.py tests/test_sign_c.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e2e_d2h_parity.log 2>&1
rc=$?; tail -2 gpurun_out/e2e_d2h_parity.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/e2e_d2h_ab.txt
for r in 1 2; do
  for mode in 0 1; do
    NET2_SHA2_D2H_COPY=$mode timeout -k 10 120 python bench.py --config e2e --steps 10 --warmup 3 > gpurun_out/e2e_ab_run.log 2>&1 || { cat gpurun_out/e2e_ab_run.log; exit 1; }
    tail -1 gpurun_out/e2e_ab_run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r d2h_copy=$mode', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms', d['h2d_GBps_per_gpu'], 'GB/s')" >> gpurun_out/e2e_d2h_ab.txt
  done
done
cat gpurun_out/e2e_d2h_ab.txt
