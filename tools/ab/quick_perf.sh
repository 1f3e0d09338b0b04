#!/bin/bash
# Quick GPU check after an arithmetic change: a parity subset, then one bench line per
# workload (summary lines in gpurun_out/quick_perf.txt).  Each GPU step has its own limit;
# the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/quick_perf.txt
: > "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${TESTS:-golden or ragged or mixed or aggregate_verify_batch or one_lane or mainnet}" > gpurun_out/quick_tests.log 2>&1 \
  || { tail -30 gpurun_out/quick_tests.log; exit 1; }
tail -2 gpurun_out/quick_tests.log
for w in ${WORKLOADS:-epoch_replay_cold mainnet_block gossip_verify deposit_av}; do
  timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-rlc \
    --no-extra-legs ${BENCH_ARGS:-} > gpurun_out/quick_$w.log 2>&1 || { tail -5 gpurun_out/quick_$w.log; exit 1; }
  python - "$w" >> "$out" <<'PY'
import json, sys
w = sys.argv[1]
d = [json.loads(l) for l in open(f"gpurun_out/quick_{w}.log") if l.startswith("{")][0]
extra = {k: d[k] for k in ("block_latency_ms",) if k in d}
ka = d.get("kernels_avg_ms") or d.get("roofline", {}).get("other_kernels_avg_ms")
print(w, "value=%.1f" % d["value"], d["unit"], "ms=%.3f" % d["ms_per_step"], "warm=%s" % d.get("warm", {}).get("value"),
      "ok=%s" % d.get("verdicts_ok"), extra, ka)
PY
  tail -1 "$out"
done
