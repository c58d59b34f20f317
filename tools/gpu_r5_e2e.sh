set -u
mkdir -p gpurun_out
for k in tx rx; do
  NET2_SHA2_DEBUG_TIMING=1 timeout -k 10 200 python tools/burst_e2e.py $k pinned > gpurun_out/burst_e2e_$k.json 2> gpurun_out/burst_e2e_$k.err || exit 1
done
for k in tx rx; do cat gpurun_out/burst_e2e_$k.json; grep 'net2 burst' gpurun_out/burst_e2e_$k.err | tail -24; done
