set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_burst_host.py tests/test_gpu_packet.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_bursts.log 2>&1 || { tail -30 gpurun_out/gputest_bursts.log; exit 1; }
tail -2 gpurun_out/gputest_bursts.log
for k in tx rx; do for m in pinned pageable; do
  NET2_SHA2_DEBUG_TIMING=1 timeout -k 10 200 python tools/burst_e2e.py $k $m > gpurun_out/burst_e2e_${k}_$m.json 2> gpurun_out/burst_e2e_${k}_$m.err || exit 1
done; done
for k in tx rx; do for m in pinned pageable; do python3 -c "import json; d=json.load(open('gpurun_out/burst_e2e_${k}_$m.json')); print('$k $m', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms', d['h2d_GBps'], 'GB/s')"; grep 'net2 burst' gpurun_out/burst_e2e_${k}_$m.err | tail -4; done; done
timeout -k 10 300 python tools/stream_ab.py --configs c3,c3_512,c2 --modes 1,2 --alternations 3 --steps 100 > gpurun_out/stream_ab_r5.txt 2>&1 || { tail gpurun_out/stream_ab_r5.txt; exit 1; }
cat gpurun_out/stream_ab_r5.txt
