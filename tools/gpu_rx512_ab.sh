# A/B: RX packing per ~512 datagrams (rx512) against per ~1 K (rx1k, shipped);
# host bursts of 256 ... 16,384 datagrams, three alternations, one call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
  if [ $((rep % 2)) = 1 ]; then order="rx1k rx512"; else order="rx512 rx1k"; fi
  for lib in $order; do
    NET2_SHA2_LIB=$PWD/tools/ab/$lib.so timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 256,1024,2048,4096,16384 --no-oracle --out gpurun_out/rx512_${lib}_$rep.jsonl > gpurun_out/rx512_${lib}_$rep.log 2>&1 || exit 1
  done
done
exit 0
