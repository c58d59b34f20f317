# A/B of library builds through bench.py: alternates the in-tree library
# with each tools/ab/*.so (NET2_SHA2_LIB), same box, same process shape.
set -u
mkdir -p gpurun_out
: > gpurun_out/ab_lib.txt
# The library run second in a pair measured ~1 % faster on some boxes
# (profiles/round2/var_drain_ab.txt), so the order flips every repetition.
for r in ${REPS:-1 2}; do
  libs="default $(ls tools/ab/*.so)"
  [ $((r % 2)) -eq 0 ] && libs=$(echo $libs | tr ' ' '\n' | tac | tr '\n' ' ')
  for c in ${CFGS:-c2 c3 hmac hmac_mtu}; do
    for lib in $libs; do
      if [ "$lib" = default ]; then unset NET2_SHA2_LIB; else export NET2_SHA2_LIB_ALLOW_OLD_ABI=1 NET2_SHA2_LIB=$PWD/$lib; fi
      timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --no-extras --steps 50 --warmup 10 > gpurun_out/ab_lib_run.log 2>&1 || { cat gpurun_out/ab_lib_run.log; exit 1; }
      tail -1 gpurun_out/ab_lib_run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r $c $(basename $lib)', round(d['value']/1e9,4), d['roofline']['kernel_ms'], d['gpu']['host'], d['gpu']['pci'])" >> gpurun_out/ab_lib.txt
    done
  done
done
cat gpurun_out/ab_lib.txt
