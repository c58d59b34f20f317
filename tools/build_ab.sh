#!/bin/bash
# Build an A/B variant of libnet2_sha2.so: tools/ab/<name>.so from
# sha2_kernels.hip compiled with the given -D flags, linked with the
# in-tree shim objects (make -C ilias_net2_amd/csrc first).
#   tools/build_ab.sh a1pf0 -DNET2_VAR_A1_PREFETCH=0
set -eu
name=$1; shift
HERE=$(cd "$(dirname "$0")" && pwd)
SRC=$HERE/../ilias_net2_amd/csrc
mkdir -p $HERE/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden \
    -Wall -Wno-unused-result -cuid=net2sha2 "$@" -c ${KSRC:-$SRC/sha2_kernels.hip} -o $HERE/ab/$name.o
# build id: hash of the device code, as the Makefile stamps it
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$HERE/ab/$name.fatbin \
    $HERE/ab/$name.o $HERE/ab/$name.tmp.o && rm -f $HERE/ab/$name.tmp.o
ID=$(sha256sum $HERE/ab/$name.fatbin | cut -c1-16)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fvisibility=hidden -DNET2_KERNEL_BUILD_ID="\"$ID\"" \
    -c $SRC/sha2_buildid.cpp -o $HERE/ab/$name.bid.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $HERE/ab/$name.so \
    $HERE/ab/$name.o $HERE/ab/$name.bid.o $SRC/build/sha2_shim.o $SRC/build/sha2_coalesce.o \
    $SRC/build/sha2_stream.o -lpthread
rm -f $HERE/ab/$name.o $HERE/ab/$name.bid.o $HERE/ab/$name.fatbin
echo built $HERE/ab/$name.so "(build id $ID)"
