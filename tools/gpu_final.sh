# Round-end refresh on one box: rocprofv3 trace + PMC passes per config,
# folded into profiles/pmc_<cfg>.json (box copy, so bench.py reports them),
# then the GPU test suite and every bench config.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUND=${ROUND:-round2}
PC="${PCFGS:-c2 c4 c3 c3_512 hmac hmac_mtu hmac512 hmac512_mtu hmac_verify_mtu hmac512_verify_mtu burst_rx burst_tx}"
CFGS="$PC" bash tools/gpu_profile.sh
rc=$?; echo "profile rc=$rc"; [ $rc -ne 0 ] && exit $rc
mkdir -p gpurun_out/profiles_$ROUND
for c in $PC; do
  python3 tools/pmc_summary.py --cfg $c --round $ROUND > /dev/null || exit 1
  cp profiles/pmc_$c.json gpurun_out/pmc_$c.json
  cp profiles/$ROUND/kernel_stats_$c.csv gpurun_out/profiles_$ROUND/ 2>/dev/null
done
bash tools/gpu_bench_all.sh
