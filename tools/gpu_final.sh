# Round-end refresh on one box: rocprofv3 trace + PMC passes per config,
# folded into profiles/pmc_<cfg>.json (box copy, so bench.py reports them),
# then the GPU test suite and every bench config.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
CFGS="${PCFGS:-c2 c4 c3 hmac}" bash tools/gpu_profile.sh
rc=$?; echo "profile rc=$rc"; [ $rc -ne 0 ] && exit $rc
for c in ${PCFGS:-c2 c4 c3 hmac}; do
  python3 tools/pmc_summary.py --cfg $c > /dev/null || exit 1
  cp profiles/pmc_$c.json gpurun_out/pmc_$c.json
done
bash tools/gpu_bench_all.sh
