# Round 4: unaligned-load probe, parity of the one-path / LDS feed-forward /
# 5-wave build, then the library A/B on the SHA-512 variable-length configs.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/unaligned_probe > gpurun_out/unaligned_probe.json
rc=$?; echo "probe rc=$rc"; cat gpurun_out/unaligned_probe.json; [ $rc -ne 0 ] && exit $rc
for v in ${ABLIBS:-onestl5}; do
  NET2_SHA2_LIB=$PWD/tools/ab/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_packet.py tests/test_gpu_dgram.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -2 gpurun_out/gputest_$v.log; [ $rc -ne 0 ] && exit $rc
done
CFGS=${CFGS:-"c3_512 hmac512_mtu hmac512_verify_mtu burst_rx burst_tx c4 c3"} REPS=${REPS:-"1 2"} bash tools/gpu_ab_lib.sh
