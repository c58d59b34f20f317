#!/bin/bash
# Ratio of the CPU port (oracle/sha2_oracle.c, what bench.py's
# cpu_baseline times on the GPU box) to the reference's own src/sha2.c, on
# identical C2 / C3 / C4 batches, both transform forms, one thread and every
# container thread.  Build container only (needs /root/reference); builds
# into a temp directory; nothing of it is committed but the JSON it writes.
#   bash tools/sha2c_ratio.sh [out.json]
set -eu
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/.." && pwd)
REF=/root/reference
OUT=${1:-$ROOT/profiles/round3/sha2c_ratio.json}
[ -f $REF/src/sha2.c ] || { echo "no reference tree" >&2; exit 2; }
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
# -O3: the reference's Release flags (CMakeLists.txt:360-363); the port is
# built the same way oracle/Makefile builds it.
for form in rolled unrolled; do
  D=""; [ $form = unrolled ] && D=-DSHA2_UNROLL_TRANSFORM
  gcc -O3 -std=gnu99 -w $D -iquote $ROOT/include/net2 -c $REF/src/sha2.c -o $T/sha2_$form.o
  gcc -O3 -std=c11 -w -c $ROOT/oracle/sha2_oracle.c -o $T/oracle.o
  gcc -O3 -std=gnu99 -Wall $D -iquote $ROOT/include/net2 -I $ROOT/oracle \
      $HERE/sha2c_ratio.c $T/sha2_$form.o $T/oracle.o -lpthread -o $T/ratio_$form
done
NT=$(nproc)
mkdir -p "$(dirname "$OUT")"
{
  echo "{\"host\": \"$(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2 | sed 's/^ //')\", \"nproc\": $NT, \"gcc\": \"$(gcc -dumpfullversion)\", \"rows\": ["
  first=1
  for cfg in c2 c3 c4; do
    for form in rolled unrolled; do
      for t in 1 $NT; do
        n=$((t == 1 ? 65536 : 262144))
        pin=""; [ $t = 1 ] && pin="taskset -c 2"
        row=$($pin $T/ratio_$form $cfg $n $t 7)
        [ $first = 1 ] && first=0 || echo ","
        echo "  $row"
      done
    done
  done
  echo "]}"
} > "$OUT"
python3 - "$OUT" <<'EOF'
import json, math, sys
d = json.load(open(sys.argv[1]))
assert all(r["digests_identical"] for r in d["rows"]), "digest mismatch"
# the constant bench.py quotes: the port's batch entry (what cpu_baseline
# times) over src/sha2.c, geometric mean over configs, forms, thread counts
rs = [r["port_batch_over_ref"] for r in d["rows"]]
d["summary"] = {"port_batch_over_sha2c_geomean": round(math.exp(sum(map(math.log, rs)) / len(rs)), 3),
                "min": min(rs), "max": max(rs), "rows": len(rs),
                "note": "spread is the shared build container's noise (alternating best-of-7 timing); "
                        "both compute identical digests"}
json.dump(d, open(sys.argv[1], "w"), indent=1)
print("summary", d["summary"])
for r in d["rows"]:
    print(f'{r["config"]} {r["form"]:8s} {r["threads"]:3d} thr  sha2.c {r["ref_sha2c_digests_per_s"]/1e6:7.3f} M/s  '
          f'port {r["port_digests_per_s"]/1e6:7.3f} M/s  (batch entry {r["port_batch_digests_per_s"]/1e6:7.3f})  '
          f'port/sha2.c {r["port_over_ref"]:.3f} / {r["port_batch_over_ref"]:.3f}')
EOF
