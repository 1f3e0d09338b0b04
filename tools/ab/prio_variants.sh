#!/bin/bash
# A/B of wave-priority builds (MBLS_G2_PRIO / MBLS_KEY_PRIO, mbls_kernels.h) on the cold epoch
# (warm leg included) and the gossip / mainnet-block / deposit workloads.  Variant libraries
# are built beforehand on the CPU:
#   make -C lambda_ethereum_consensus_amd/csrc OBJ=../build_gXkY OUT=../lib/var_gXkY \
#        CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -DMBLS_G2_PRIO=X -DMBLS_KEY_PRIO=Y"
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/prio_variants.txt
: > "$out"
run() {  # name lib workload
  local lib=$2
  [ "$lib" = default ] && lib=lambda_ethereum_consensus_amd/lib/libmbls.so || lib=lambda_ethereum_consensus_amd/lib/var_$2/libmbls.so
  local line
  line=$(MBLS_LIB_PATH=$lib timeout -k 10 240 python bench.py --workload "$3" --steps ${STEPS:-50} --warmup 2 \
         --no-cpu-baseline --no-rlc --no-extra-legs 2>gpurun_out/prio_err.log | grep '^{') || { echo "$1 $3 failed"; tail -5 gpurun_out/prio_err.log; return 1; }
  python - "$1" "$3" "$line" >> "$out" <<'EOF'
import json, sys
d = json.loads(sys.argv[3])
w = d.get("warm", {})
print(sys.argv[1], sys.argv[2], "value=%.1f" % d["value"], "ms=%.3f" % d["ms_per_step"],
      "roof_ms=%s" % d.get("roofline", {}).get("avg_launch_ms"), "warm=%s" % w.get("value"))
EOF
  tail -1 "$out"
}
for v in ${VARIANTS:-default g0k0 g0k2 g1k2 g3k3}; do
  for w in ${WORKLOADS:-epoch_replay_cold gossip_verify}; do
    run "$v" "$v" "$w" || exit 1
  done
done
