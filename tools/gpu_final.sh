# Round-end refresh on one box: rocprofv3 trace + PMC passes per config,
# folded into profiles/pmc_<cfg>.json (box copy, so bench.py reports them),
# then the GPU test suite and every bench config.
set -u
ROUND=${ROUND:-round3} bash tools/gpu_profile_round.sh || exit 1
bash tools/gpu_bench_all.sh
