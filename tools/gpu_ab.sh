# In-process A/B of kernel build variants on one box: each binary runs the
# same variant table; alternating runs bound the run-to-run drift.
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for b in ${AB_BINS:-kernel_ab kernel_ab_u2}; do
    timeout -k 10 200 ./tools/$b > gpurun_out/ab256_${b}_$r.json 2>&1 || exit $?
  done
  for b in ${AB512_BINS:-kernel_ab kernel_ab_shr}; do
    AB512=1 timeout -k 10 200 ./tools/$b > gpurun_out/ab512_${b}_$r.json 2>&1 || exit $?
  done
done
exit 0
