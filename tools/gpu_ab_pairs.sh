# A/B of library builds through bench.py, one config at a time with its own
# list of builds: PAIRS="cfg:libA,libB,... cfg2:..." (lib = default for the
# in-tree library, else tools/ab/<lib>.so), the build order flipped every
# repetition (REPS, default "1 2"); one line per run into
# gpurun_out/ab_pairs.txt: rep config lib G/s kernel_ms sclk host pci.
set -u
mkdir -p gpurun_out
: > gpurun_out/ab_pairs.txt
for r in ${REPS:-1 2}; do
  for pair in $PAIRS; do
    c=${pair%%:*}
    libs=$(echo ${pair#*:} | tr ',' ' ')
    [ $((r % 2)) -eq 0 ] && libs=$(echo $libs | tr ' ' '\n' | tac | tr '\n' ' ')
    for lib in $libs; do
      if [ "$lib" = default ]; then unset NET2_SHA2_LIB; else export NET2_SHA2_LIB_ALLOW_OLD_ABI=1 NET2_SHA2_LIB=$PWD/tools/ab/$lib.so; fi
      timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --no-extras --steps ${STEPS:-50} --warmup 10 > gpurun_out/ab_run.log 2>&1 || { cat gpurun_out/ab_run.log; exit 1; }
      tail -1 gpurun_out/ab_run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r $c $lib', round(d['value']/1e9,4), d['roofline']['kernel_ms'], d['gpu'].get('sclk_mhz_during_timed_steps'), d['gpu']['host'], d['gpu']['pci'])" >> gpurun_out/ab_pairs.txt
    done
  done
  cat gpurun_out/ab_pairs.txt
done
