export PAIRS="hmac512:default,hfglds,r4base burst_rx:default,r4base hmac512_verify_mtu:default,r4base hmac512_mtu:default,r4base burst_tx:default,r4base c3:default,r4base c3_512:default,r4base hmac_mtu:default,r4base"
REPS="1 2" bash tools/gpu_ab_pairs.sh
