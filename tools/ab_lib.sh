#!/bin/bash
# A/B of library variants (tools/build_variant.sh) on the default bench workload: one summary line
# per (rep, variant) with the cold headline, the warm leg and its kernels' per-launch times, in
# gpurun_out/ab_lib.txt.  VARIANTS are directory names under lambda_ethereum_consensus_amd/lib
# ("-" = the in-tree build), interleaved REPS times.  Every GPU step has its own time limit and
# the chain stops at the first failure.
#   VARIANTS="- var_x1 var_xall" STEPS=100 REPS=2 bash tools/ab_lib.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/ab_lib.txt
: > "$out"
for rep in $(seq 1 ${REPS:-1}); do
  for v in ${VARIANTS:--}; do
    lib=""
    [ "$v" != "-" ] && lib="lambda_ethereum_consensus_amd/lib/$v/libmbls.so"
    line=$(MBLS_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload ${WORKLOAD:-epoch_replay_cold} \
           --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs 2>gpurun_out/ab_lib_err.log \
           | grep '^{') || { echo "$v failed"; tail -5 gpurun_out/ab_lib_err.log; exit 1; }
    python3 - "$rep" "$v" "$line" >> "$out" <<'EOF'
import json, sys
d = json.loads(sys.argv[3])
w = d.get("warm") or {}
wr = w.get("roofline") or {}
ks = {k: v.get("avg_launch_ms") for k, v in (wr.get("kernels") or {}).items()}
print("rep%s %-10s cold=%.1f warm=%s chip_frac=%s warm_ms=%s kernels=%s ok=%s/%s" % (
    sys.argv[1], sys.argv[2], d["value"], w.get("value"), wr.get("chip_frac"), w.get("ms_per_step"), ks,
    d.get("verdicts_ok"), w.get("verdicts_ok")))
EOF
    tail -1 "$out"
  done
done
