export PAIRS="hmac512:default,hfnoglds,r4base burst_rx:default,r4base hmac512_verify_mtu:default,r4base hmac512_mtu:default,r4base burst_tx:default,r4base hmac_mtu:default,r4base hmac:default,r4base hmac_verify_mtu:default,r4base"
REPS="1 2" bash tools/gpu_ab_pairs.sh > /dev/null && cp gpurun_out/ab_pairs.txt gpurun_out/ab_pairs2.txt &&
unset NET2_SHA2_LIB && timeout -k 10 400 python bench.py > gpurun_out/bench_default_r5a.json 2> gpurun_out/bench_default_r5a.err &&
bash tools/gpu_burst_bins.sh > /dev/null; rc=$?
cat gpurun_out/ab_pairs2.txt; tail -c 2500 gpurun_out/bench_default_r5a.json; tail -3 gpurun_out/bench_default_r5a.err; cat gpurun_out/burst_bins.txt; exit $rc
