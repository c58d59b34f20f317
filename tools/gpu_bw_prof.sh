# Kernel durations of the small-burst form, by library build and burst size:
# tools/burst_sizes.py under rocprofv3 --kernel-trace --stats, one process
# per (build, size).  LIBS: default or tools/ab/<name>.so.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in ${LIBS:-default v1}; do
  for n in ${SIZES:-64 1024}; do
    if [ "$lib" = default ]; then unset NET2_SHA2_LIB; else export NET2_SHA2_LIB_ALLOW_OLD_ABI=1 NET2_SHA2_LIB=$PWD/tools/ab/$lib.so; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/bwp_${lib}_$n -o run --output-format csv -- python3 tools/burst_sizes.py --sizes $n --no-oracle > gpurun_out/bwp_${lib}_$n.log 2>&1 || exit 1
    rm -f gpurun_out/bwp_${lib}_$n/run_kernel_trace.csv
  done
done
