# The G form with every lane of wave 0 on a datagram slot (v3) against the
# shipped one-datagram-per-workgroup form (default): parity (every wave-form
# test, under NET2_SHA2_LIB), kernel durations by size, and end-to-end burst
# calls, order flipped.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
NET2_SHA2_LIB_ALLOW_OLD_ABI=1 NET2_SHA2_LIB=$PWD/tools/ab/v3.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_burst_wave.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bw3_tests.log 2>&1 || exit 1
LIBS="default v3" SIZES="64 1024 4096" bash tools/gpu_bw_prof.sh || exit 1
for rep in 1 2; do
  libs="default v3"; [ $rep -eq 2 ] && libs="v3 default"
  for lib in $libs; do
    if [ "$lib" = default ]; then unset NET2_SHA2_LIB; else export NET2_SHA2_LIB_ALLOW_OLD_ABI=1 NET2_SHA2_LIB=$PWD/tools/ab/$lib.so; fi
    NET2_BURST_WAVE_MAX=$([ "$lib" = v3 ] && echo 16384 || echo 1024) timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 64,1024,2048,4096,8192,16384 --no-oracle --out gpurun_out/bw3_${lib}_$rep.jsonl > gpurun_out/bw3_${lib}_$rep.log 2>&1 || exit 1
  done
done
