# A/B: RX packs with a thread per ~1 K datagrams, TX per ~4 K (rxpack1k)
# against both per ~4 K (pack4k), libraries under tools/ab/; host bursts of
# 4,096 ... 65,536 datagrams, three alternations in flipped order, one call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
  if [ $((rep % 2)) = 1 ]; then order="pack4k rxpack1k"; else order="rxpack1k pack4k"; fi
  for lib in $order; do
    NET2_SHA2_LIB=$PWD/tools/ab/$lib.so timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 4096,16384,65536 --no-oracle --out gpurun_out/pack2_${lib}_$rep.jsonl > gpurun_out/pack2_${lib}_$rep.log 2>&1 || exit 1
  done
done
exit 0
