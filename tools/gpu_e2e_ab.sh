# A/B of host-path library builds through tools/e2e_host.py: alternates the
# in-tree library with each tools/ab/*.so (NET2_SHA2_LIB) on one box.
set -u
mkdir -p gpurun_out
: > gpurun_out/e2e_ab.txt
for r in 1 2 3; do
  for lib in default tools/ab/*.so; do
    if [ "$lib" = default ]; then unset NET2_SHA2_LIB; else export NET2_SHA2_LIB=$PWD/$lib; fi
    timeout -k 10 120 python -u tools/e2e_host.py > gpurun_out/e2e_ab_run.log 2>&1 || { cat gpurun_out/e2e_ab_run.log; exit 1; }
    grep -E "GB/s" gpurun_out/e2e_ab_run.log | sed "s|^|$r $(basename $lib): |" >> gpurun_out/e2e_ab.txt
  done
done
cat gpurun_out/e2e_ab.txt
