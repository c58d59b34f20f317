# A/B: pack-pool workers spinning only after a job they took part in
# (spinpart) against every worker spinning after every job (spinall),
# libraries under tools/ab/: host bursts of 1 K ... 1 M datagrams (call
# time) and the per-thread CPU of 1 M-datagram calls, three alternations in
# flipped order, one call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
  if [ $((rep % 2)) = 1 ]; then order="spinall spin50"; else order="spin50 spinall"; fi
  for lib in $order; do
    NET2_SHA2_LIB=$PWD/tools/ab/$lib.so timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 1024,4096,65536,1048576 --no-oracle --out gpurun_out/spin_${lib}_$rep.jsonl > gpurun_out/spin_${lib}_$rep.log 2>&1 || exit 1
    NET2_SHA2_LIB=$PWD/tools/ab/$lib.so REPS=10 timeout -k 10 100 python3 -u tools/burst_debug_timing.py > gpurun_out/spin_cpu_${lib}_$rep.txt 2>&1 || exit 1
  done
done
exit 0
