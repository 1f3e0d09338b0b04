#!/bin/bash
# Per-kernel register / scratch metadata of the gfx950 code objects in the built objects:
#   tools/kernel_meta.sh [obj ...]   (default: every lambda_ethereum_consensus_amd/build/mbls_k_*.o)
# Prints name, arch VGPRs, AGPRs, SGPRs, private segment (scratch) bytes per lane, spill counts.
set -e -o pipefail
LLVM=/opt/rocm/lib/llvm/bin
cd "$(dirname "$0")/.."
objs=("$@")
[ ${#objs[@]} -eq 0 ] && objs=(lambda_ethereum_consensus_amd/build/mbls_k_*.o)
tmp=$(mktemp -d)
for o in "${objs[@]}"; do
  b=$(basename "$o" .o)
  # an explicit output file: llvm-objcopy with only an input rewrites it in place (and makes
  # every object newer than libmbls.so)
  $LLVM/llvm-objcopy --dump-section=.hip_fatbin="$tmp/$b.fatbin" "$o" "$tmp/$b.copy.o"
  $LLVM/clang-offload-bundler --unbundle --type=o --input="$tmp/$b.fatbin" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$tmp/$b.co"
  $LLVM/llvm-readelf --notes "$tmp/$b.co" | python3 "$(dirname "$0")/kernel_meta.py"
done
rm -rf "$tmp"
