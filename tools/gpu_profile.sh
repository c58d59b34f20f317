# rocprofv3 passes for the bench configs: one kernel-trace/stats pass and
# separate PMC passes (never combined with tracing), per config.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
CFGS=${CFGS:-"c2 c4 c3"}
for c in $CFGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --no-extras --steps 20 > gpurun_out/prof_$c.log 2>&1
  rc=$?; echo "trace $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  for pass in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
    tag=$(echo $pass | cut -d' ' -f1)
    timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/pmc_${c}_$tag -o run -- python3 bench.py --config $c --steps 5 --warmup 2 --prewarm-ms 500 --no-cpu-baseline --no-extras > gpurun_out/pmc_${c}_$tag.log 2>&1
    rc=$?; echo "pmc $c $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
