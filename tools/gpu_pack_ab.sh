# A/B: host pack threads per ~1 K datagrams (pack1k) against per ~4 K
# (pack4k, the build before), libraries under tools/ab/; host bursts of
# 1,024 ... 65,536 datagrams, three alternations in flipped order, one call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
  if [ $((rep % 2)) = 1 ]; then order="pack4k pack1k"; else order="pack1k pack4k"; fi
  for lib in $order; do
    NET2_SHA2_LIB=$PWD/tools/ab/$lib.so timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 1024,2048,4096,8192,16384,65536 --no-oracle --out gpurun_out/pack_${lib}_$rep.jsonl > gpurun_out/pack_${lib}_$rep.log 2>&1 || exit 1
  done
done
exit 0
