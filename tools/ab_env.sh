#!/bin/bash
# A/B of engine environment knobs on bench workloads, one JSON summary line per
# (setting, workload) in gpurun_out/ab_env.txt.  SETTINGS is a space-separated list of
# comma-joined VAR=VALUE groups ("-" = defaults), e.g.
#   SETTINGS="- MBLS_KEY_STREAMS=2" WORKLOADS="epoch_replay_cold gossip_verify" bash tools/ab_env.sh
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/ab_env.txt
: > "$out"
for rep in $(seq 1 ${REPS:-1}); do
for s in ${SETTINGS:--}; do
  for w in ${WORKLOADS:-epoch_replay_cold}; do
    envs=()
    [ "$s" != "-" ] && IFS=, read -r -a envs <<< "$s"
    line=$(env "${envs[@]}" timeout -k 10 240 python bench.py --workload "$w" --steps ${STEPS:-50} --warmup 2 \
           --no-cpu-baseline --no-rlc --no-extra-legs ${BENCH_ARGS:-} 2>gpurun_out/ab_err.log | grep '^{') \
      || { echo "$s $w failed"; tail -5 gpurun_out/ab_err.log; exit 1; }
    python - "$s" "$w" "$line" >> "$out" <<'EOF'
import json, sys
d = json.loads(sys.argv[3])
w = d.get("warm") or {}
print(sys.argv[1], sys.argv[2], "value=%.1f" % d["value"], "ms=%.3f" % d["ms_per_step"],
      "roof_ms=%s" % d.get("roofline", {}).get("avg_launch_ms"), "warm=%s" % w.get("value"),
      "ok=%s" % d.get("verdicts_ok"), "block_latency_ms=%s" % d.get("block_latency_ms"),
      "kernels=%s" % d.get("kernels_avg_ms"))
EOF
    tail -1 "$out"
  done
done
done
