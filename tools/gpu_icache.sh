# Instruction-cache counters per bench config (one --pmc pass per pair,
# never combined with tracing), then a median-per-launch summary of the
# config's kernel.  CFGS selects the configs; NET2_SHA2_LIB an A/B build.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CFGS:-c4 burst_rx}; do
  for pass in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQ_IFETCH SQ_WAVES"; do
    tag=$(echo $pass | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/ic_${c}_$tag -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --prewarm-ms 100 --no-cpu-baseline --no-extras > gpurun_out/ic_${c}_$tag.log 2>&1
    rc=$?; echo "pmc $c $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
python3 tools/icache_summary.py ${CFGS:-c4 burst_rx}
