# A/B: zero-copy for every single-chunk keyed host burst (zcbig, NET2_BURST_ZC_MAX
# 131072 without the one-launch condition) against the shipped rule (zc: only
# the one-launch form), host bursts of 16,385 ... 1 M datagrams, three
# alternations in flipped order, one call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
true
for rep in 1 2 3; do
  if [ $((rep % 2)) = 1 ]; then order="zc zcbig"; else order="zcbig zc"; fi
  for lib in $order; do
    NET2_SHA2_LIB=$PWD/tools/ab/$lib.so timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 16385,32768,65536,131072,1048576 --no-oracle --out gpurun_out/zcbig_${lib}_$rep.jsonl > gpurun_out/zcbig_${lib}_$rep.log 2>&1 || exit 1
  done
done
exit 0
