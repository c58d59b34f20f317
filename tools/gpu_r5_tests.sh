mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_r5a.log 2>&1
rc=$?
tail -30 gpurun_out/gputest_r5a.log
exit $rc
