# Host-path A/B: a library build (tools/ab/$LIB.so) against the in-tree one,
# alternated: host burst e2e (tools/burst_e2e.py, pinned and pageable, RX
# and TX) and the variable-layout digest e2e (tools/e2e_var.py).
set -u
mkdir -p gpurun_out
: > gpurun_out/meta_ab.txt
for r in ${REPS:-1 2}; do
  libs="${LIB:-pairall} default"; [ $((r % 2)) -eq 0 ] && libs="default ${LIB:-pairall}"
  for l in $libs; do
    if [ $l = default ]; then unset NET2_SHA2_LIB; else export NET2_SHA2_LIB=$PWD/tools/ab/$l.so; fi
    [ -n "${NO_BURST:-}" ] || for k in tx rx; do for m in pinned pageable; do
      timeout -k 10 120 python tools/burst_e2e.py $k $m > gpurun_out/be2e.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/be2e.json').read().strip().splitlines()[-1]); print('$r $l $k $m', round(d['value']/1e6,2), d['ms_per_step'])" >> gpurun_out/meta_ab.txt
    done; done
    for m in pageable pinned; do
      timeout -k 10 300 python tools/e2e_var.py $m > gpurun_out/e2e_var.txt 2>&1 || exit 1
      echo "$r $l $(tail -1 gpurun_out/e2e_var.txt)" >> gpurun_out/meta_ab.txt
    done
  done
done
cat gpurun_out/meta_ab.txt
