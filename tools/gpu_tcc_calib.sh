#!/bin/bash
# Read-request accounting of the L2 (TCC) by request size, for C2 (a
# known 1 GiB stream: the calibration) and the variable-length configs.
# One rocprofv3 pass per counter group (at most 4 TCC counters a pass),
# never combined with tracing.  Summarised by tools/tcc_summary.py.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
CFGS=${CFGS:-"c2 c3"}
for c in $CFGS; do
  for pass in "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_BUBBLE" \
              "TCC_EA0_RDREQ_DRAM TCC_EA0_RDREQ_DRAM_32B TCC_READ_SECTORS TCC_MISS"; do
    tag=$(echo $pass | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/tcc_${c}_$tag -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --prewarm-ms 100 --no-cpu-baseline --no-extras > gpurun_out/tcc_${c}_$tag.log 2>&1
    rc=$?; echo "tcc $c $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
