# A/B: pack-pool participants spinning 100 us after a job and TX packing per
# ~1 K datagrams too (spin100) against the shipped 500 us / TX per ~4 K (cur),
# libraries under tools/ab/; 1,024 ... 1 M datagrams, three alternations.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
  if [ $((rep % 2)) = 1 ]; then order="cur spin100"; else order="spin100 cur"; fi
  for lib in $order; do
    NET2_SHA2_LIB=$PWD/tools/ab/$lib.so timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 1024,4096,16384,65536,1048576 --no-oracle --out gpurun_out/spin100_${lib}_$rep.jsonl > gpurun_out/spin100_${lib}_$rep.log 2>&1 || exit 1
  done
done
exit 0
