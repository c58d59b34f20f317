set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_burst_host.py tests/test_gpu_packet.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_bursts.log 2>&1 || { tail -30 gpurun_out/gputest_bursts.log; exit 1; }
tail -2 gpurun_out/gputest_bursts.log
for k in tx rx; do
  NET2_SHA2_DEBUG_TIMING=1 timeout -k 10 200 python tools/burst_e2e.py $k pinned > gpurun_out/burst_e2e_$k.json 2> gpurun_out/burst_e2e_$k.err || exit 1
done
for k in tx rx; do cat gpurun_out/burst_e2e_$k.json; grep 'net2 burst' gpurun_out/burst_e2e_$k.err | tail -6; done
