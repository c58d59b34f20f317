# A/B: small keyed host bursts read through the host mapping by their kernel
# (zc) against two copies first (copy), libraries under tools/ab/; the burst
# GPU tests on the in-tree library (zc) first, then host bursts of 64 ... 16,384 datagrams, three
# alternations in flipped order, one call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_burst_host.py tests/test_gpu_burst_wave.py tests/test_gpu_failures.py -x -q --timeout 120 --timeout-method thread > gpurun_out/zc_tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  if [ $((rep % 2)) = 1 ]; then order="copy zc"; else order="zc copy"; fi
  for lib in $order; do
    NET2_SHA2_LIB=$PWD/tools/ab/$lib.so timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 64,256,1024,2048,4096,8192,16384 --no-oracle --out gpurun_out/zc_${lib}_$rep.jsonl > gpurun_out/zc_${lib}_$rep.log 2>&1 || exit 1
  done
done
exit 0
