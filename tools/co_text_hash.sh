#!/bin/bash
# sha256 of the .text section of each object's gfx950 code object (instruction identity of two
# builds of the same source, e.g. before / after deleting dead compile-time branches):
#   tools/co_text_hash.sh [obj ...]   (default: lambda_ethereum_consensus_amd/build/mbls_k_*.o)
set -e -o pipefail
LLVM=/opt/rocm/lib/llvm/bin
cd "$(dirname "$0")/.."
objs=("$@")
[ ${#objs[@]} -eq 0 ] && objs=(lambda_ethereum_consensus_amd/build/mbls_k_*.o)
tmp=$(mktemp -d)
for o in "${objs[@]}"; do
  b=$(basename "$o" .o)
  $LLVM/llvm-objcopy --dump-section=.hip_fatbin="$tmp/$b.fatbin" "$o" "$tmp/$b.copy.o"
  $LLVM/clang-offload-bundler --unbundle --type=o --input="$tmp/$b.fatbin" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$tmp/$b.co"
  $LLVM/llvm-objcopy -O binary --only-section=.text "$tmp/$b.co" "$tmp/$b.text"
  echo "$(sha256sum < "$tmp/$b.text" | cut -c1-16) $(stat -c %s "$tmp/$b.text") $b"
done
rm -rf "$tmp"
