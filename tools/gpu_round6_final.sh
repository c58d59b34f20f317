# Round-6 end-of-round measurements in one GPU call (outputs under
# gpurun_out/, copied into profiles/round6/ by hand):
#   1. counter summaries of the remaining configs (gpu_round_final.sh
#      STAGE=profile) -- skipped when SKIP_PROFILE=1;
#   2. the driver's default bench line;
#   3. the GPU test suite and smoke();
#   4. host bursts by size with the oracle beside them, and
#      the binning threshold A/B (NET2_BURST_BIN_MIN 4,096 against the
#      default 65,536) at the sizes it decides.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_PROFILE:-0}" != 1 ]; then
  STAGE=profile ROUND=round6 PCFGS="${PCFGS:-hmac hmac_mtu hmac512 hmac512_mtu hmac_verify_mtu hmac512_verify_mtu ph_iv}" \
    timeout -k 10 600 bash tools/gpu_round_final.sh > gpurun_out/r6_profile2.log 2>&1 || exit 1
fi
timeout -k 10 300 python3 bench.py > gpurun_out/r6_bench_default.log 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r6_final_gputest.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/burst_sizes.py --out gpurun_out/r6_burst_sizes_final.jsonl > gpurun_out/r6_burst_sizes_final.log 2>&1 || exit 1
NET2_BURST_BIN_MIN=4096 timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 4096,16384,32768 --no-oracle --out gpurun_out/r6_bs_binmin4096.jsonl > gpurun_out/r6_bs_binmin4096.log 2>&1 || exit 1
exit 0
