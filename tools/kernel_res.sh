#!/bin/bash
# VGPR / SGPR / spill counts of every kernel in the built libnet2_sha2 kernels
# object (code-object notes), optionally filtered by a name pattern.
#   bash tools/kernel_res.sh [pattern]
set -eu
B=/opt/rocm/lib/llvm/bin
OBJ=${OBJ:-$(dirname "$0")/../ilias_net2_amd/csrc/build/sha2_kernels.o}
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
$B/llvm-objcopy --dump-section=.hip_fatbin="$T/fat.bin" "$OBJ"
$B/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
    --input="$T/fat.bin" --output="$T/k.co" --unbundle
$B/llvm-readelf --notes "$T/k.co" |
  grep -E "^ +\.name:|\.vgpr_count:|\.sgpr_count:|\.vgpr_spill_count|\.private_segment_fixed_size" |
  paste - - - - - | sed 's/  */ /g' | grep -E "${1:-.}" || true
