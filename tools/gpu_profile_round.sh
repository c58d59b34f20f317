# rocprofv3 trace + PMC passes for the configs in PCFGS, folded into
# profiles/pmc_<cfg>.json (stamped with the loaded library's build id) and
# profiles/$ROUND/kernel_stats_<cfg>.csv; copies under gpurun_out/ for the
# trip back.  tools/gpu_final.sh = this + tools/gpu_bench_all.sh.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUND=${ROUND:-round3}
PC="${PCFGS:-c2 c4 c3 c3_512 hmac hmac_mtu hmac512 hmac512_mtu hmac_verify_mtu hmac512_verify_mtu burst_rx burst_tx ph_iv}"
CFGS="$PC" bash tools/gpu_profile.sh
rc=$?; echo "profile rc=$rc"; [ $rc -ne 0 ] && exit $rc
mkdir -p gpurun_out/profiles_$ROUND
for c in $PC; do
  python3 tools/pmc_summary.py --cfg $c --round $ROUND > /dev/null || exit 1
  cp profiles/pmc_$c.json gpurun_out/pmc_$c.json
  cp profiles/$ROUND/kernel_stats_$c.csv gpurun_out/profiles_$ROUND/ 2>/dev/null
done
exit 0
