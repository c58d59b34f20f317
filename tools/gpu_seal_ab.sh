# A/B: keyed host TX sealed by the kernel straight into the caller's
# page-locked buffer (seal) against records scattered by the host (scatter),
# libraries under tools/ab/; the GPU tests of the host bursts and their
# failure paths first, then host bursts of 1 K ... 1 M datagrams, three
# alternations in flipped order, one call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_failures.py tests/test_gpu_burst_host.py tests/test_gpu_burst_wave.py -x -q --timeout 120 --timeout-method thread > gpurun_out/seal_tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  if [ $((rep % 2)) = 1 ]; then order="scatter seal"; else order="seal scatter"; fi
  for lib in $order; do
    NET2_SHA2_LIB=$PWD/tools/ab/$lib.so timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 1024,4096,16384,65536,1048576 --no-oracle --out gpurun_out/seal_${lib}_$rep.jsonl > gpurun_out/seal_${lib}_$rep.log 2>&1 || exit 1
  done
done
exit 0
