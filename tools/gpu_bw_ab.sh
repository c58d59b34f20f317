set -u
mkdir -p gpurun_out
for rep in 1 2; do
  libs="default w1r48 w2r16 w1r16"
  [ $rep -eq 2 ] && libs="w1r16 w2r16 w1r48 default"
  for lib in $libs; do
    if [ "$lib" = default ]; then unset NET2_SHA2_LIB; else export NET2_SHA2_LIB_ALLOW_OLD_ABI=1 NET2_SHA2_LIB=$PWD/tools/ab/$lib.so; fi
    timeout -k 10 200 python3 -u tools/burst_sizes.py --sizes 64,1024,4096,16384 --no-oracle --out gpurun_out/bw_${lib}_$rep.jsonl > gpurun_out/bw_${lib}_$rep.log 2>&1 || exit 1
  done
done
