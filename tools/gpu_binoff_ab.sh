# Does the length binning matter on the host burst path?  (VERDICT round 5,
# item 7: a host-built bin order would drop the binning launch from host
# chunks.)  Host bursts of 64 K and 1 M datagrams with the binning as shipped
# against no binning at all (NET2_BURST_BIN_MIN above every size: the lane
# form in arrival order, ~1.8x the hash kernel's time), two repetitions in
# flipped order, one call.  If the call time does not move with binning
# switched off entirely, no cheaper bin order can move it either.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  if [ $rep = 1 ]; then order="binned off"; else order="off binned"; fi
  for v in $order; do
    if [ $v = off ]; then export NET2_BURST_BIN_MIN=1099511627776; else unset NET2_BURST_BIN_MIN; fi
    timeout -k 10 240 python3 -u tools/burst_sizes.py --sizes 65536,1048576 --no-oracle --out gpurun_out/binoff_${v}_$rep.jsonl > gpurun_out/binoff_${v}_$rep.log 2>&1 || exit 1
  done
done
unset NET2_BURST_BIN_MIN
exit 0
