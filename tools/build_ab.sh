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
# build id: the in-tree hash of the kernel sources + a hash of the -D flags
ID=$(cat $SRC/sha2_kernels.hip $SRC/sha2_device.h $SRC/sha2_launch.h | sha256sum | cut -c1-16)+$(echo "$@" | sha256sum | cut -c1-8)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden \
    -Wall -Wno-unused-result "$@" -DNET2_KERNEL_BUILD_ID="\"$ID\"" -c $SRC/sha2_kernels.hip -o $HERE/ab/$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $HERE/ab/$name.so \
    $HERE/ab/$name.o $SRC/build/sha2_shim.o $SRC/build/sha2_coalesce.o \
    $SRC/build/sha2_stream.o -lpthread
rm -f $HERE/ab/$name.o
echo built $HERE/ab/$name.so
