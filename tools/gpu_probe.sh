# Round-1 probe: VALU issue rates, gpu parity tests, PMC passes on config c2.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/valu_probe > gpurun_out/valu_probe.json 2>&1
rc=$?; echo "valu_probe rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for pass in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/pmc_c2_$tag -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/pmc_c2_$tag.log 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
