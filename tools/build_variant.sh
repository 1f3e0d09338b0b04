#!/bin/bash
# Variant library for A/B runs: rebuild the given translation units with extra flags and link
# them with the default objects into lambda_ethereum_consensus_amd/lib/var_$NAME/libmbls.so
# (loaded with MBLS_LIB_PATH).
#   tools/build_variant.sh NAME "-DFOO=1" mbls_k_lg.hip [mbls_k_g2.hip ...]
set -e -o pipefail
cd "$(dirname "$0")/../lambda_ethereum_consensus_amd/csrc"
name=$1; flags=$2; shift 2
out=../lib/var_$name; obj=../build/var_$name
mkdir -p "$out" "$obj"
objs=()
for o in mbls_k_g1 mbls_k_g2 mbls_k_pair mbls_k_pairs_av mbls_k_lg mbls_k_lg6 mbls_k_av6 mbls_k_g2w mbls_k_ssz mbls_engine mbls_pipeline mbls_scratch mbls_queue mbls_status; do objs+=("../build/$o.o"); done
for src in "$@"; do
  b=$(basename "$src"); b=${b%.*}
  hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 -munsafe-fp-atomics $flags -c "$src" -o "$obj/$b.o" &
  for i in "${!objs[@]}"; do [ "${objs[$i]}" = "../build/$b.o" ] && objs[$i]="$obj/$b.o"; done
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libmbls.so" "${objs[@]}" -lpthread -L/opt/rocm/lib -lrccl -lamdhip64 -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib
echo "built $out/libmbls.so"
