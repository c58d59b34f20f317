# A/B at the bench's TX shape (1 M MTU datagrams from pinned memory, the
# layout of bench.py's burst_tx_e2e): shipped vs txnobin, three alternations
# in flipped order, one call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
  if [ $((rep % 2)) = 1 ]; then order="shipped txnobin"; else order="txnobin shipped"; fi
  for lib in $order; do
    NET2_SHA2_LIB=$PWD/tools/ab/$lib.so timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 1048576 --no-oracle --out gpurun_out/txbin3_${lib}_$rep.jsonl > gpurun_out/txbin3_${lib}_$rep.log 2>&1 || exit 1
  done
done
exit 0
