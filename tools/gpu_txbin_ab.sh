# A/B: host TX chunks copied as they lie, hashed in arrival order (txnobin)
# against the shipped binned order (shipped), libraries from
# tools/build_ab.sh / tools/ab/; host bursts of 64 K and 1 M datagrams, two
# repetitions in flipped order, one call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  if [ $rep = 1 ]; then order="shipped txnobin"; else order="txnobin shipped"; fi
  for lib in $order; do
    NET2_SHA2_LIB=$PWD/tools/ab/$lib.so timeout -k 10 240 python3 -u tools/burst_sizes.py --sizes 65536,1048576 --no-oracle --out gpurun_out/txbin_${lib}_$rep.jsonl > gpurun_out/txbin_${lib}_$rep.log 2>&1 || exit 1
  done
done
exit 0
