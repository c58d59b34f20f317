# A/B of whole-library builds (tools/ab/*.so) on the coalescer: each build is
# linked into place as libnet2_sha2.so in a scratch directory ahead of the
# in-tree one on LD_LIBRARY_PATH; tools/coalesce_bench for 1/8/32/64 threads.
set -u
mkdir -p gpurun_out; : > gpurun_out/co_lib_ab.txt
for r in 1 2; do for lib in default tools/ab/*.so; do
  if [ "$lib" = default ]; then D=$PWD/ilias_net2_amd; else
    D=/tmp/co_ab_$(basename $lib .so); mkdir -p $D; ln -sf $PWD/$lib $D/libnet2_sha2.so; fi
  for alg in ${ALGS:-3}; do
    LD_LIBRARY_PATH=$D timeout -k 10 60 tools/coalesce_bench $alg 1024 1 1 8 32 64 > gpurun_out/co_run.jsonl || exit 1
    sed "s|^|r$r $(basename $lib) |" gpurun_out/co_run.jsonl >> gpurun_out/co_lib_ab.txt
  done
done; done
wc -l gpurun_out/co_lib_ab.txt
