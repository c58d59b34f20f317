# rocprofv3 trace + PMC passes for the configs in PCFGS, folded into
# profiles/pmc_<cfg>.json (stamped with the loaded library's build id) and
# profiles/$ROUND/kernel_stats_<cfg>.csv; copies under gpurun_out/ for the
# trip back.  tools/gpu_final.sh = this + tools/gpu_bench_all.sh.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUND=${ROUND:-round3}
PC="${PCFGS:-c2 c4 c3 c3_512 hmac hmac_mtu hmac512 hmac512_mtu hmac_verify_mtu hmac512_verify_mtu burst_rx burst_tx burst_rx256 ph_iv}"
CFGS="$PC" bash tools/gpu_profile.sh
rc=$?; echo "profile rc=$rc"; [ $rc -ne 0 ] && exit $rc
mkdir -p gpurun_out/profiles_$ROUND
for c in $PC; do
  python3 tools/pmc_summary.py --cfg $c --round $ROUND > /dev/null || exit 1
  cp profiles/pmc_$c.json gpurun_out/pmc_$c.json
  cp profiles/$ROUND/kernel_stats_$c.csv gpurun_out/profiles_$ROUND/ 2>/dev/null
done
# the raw per-dispatch CSVs are folded now: drop them (after every config is
# summarised -- pmc_hmac_* also matches pmc_hmac_mtu_*), so what comes back
# stays under gpurun's 64 MiB
for c in $PC; do
  for pass in SQ_INSTS_VALU SQ_ACTIVE_INST_VALU FETCH_SIZE WRITE_SIZE SQ_INSTS_SALU; do
    rm -rf gpurun_out/pmc_${c}_$pass
  done
  rm -f gpurun_out/prof_$c/run_kernel_trace.csv
done
exit 0
