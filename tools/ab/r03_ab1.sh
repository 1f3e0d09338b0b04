#!/bin/bash
# r03 A/B 1: aggregation stream priority (engine knob) on the cold epoch, and the lane-group
# kernels bounded to 256 registers (var_lg2) on the warm epoch and one mainnet block.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab1
mkdir -p $OUT
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-rlc --no-extra-legs"
run() {  # name env... -- args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?
  python3 - "$OUT/$name.json" "$name" <<'PY'
import json, sys
try:
    d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]
except Exception as e:
    print(sys.argv[2], "no result", e); sys.exit(0)
w = d.get("warm") or {}
print("%-22s value=%9.1f ms=%7.3f ok=%s warm=%s key_ms=%s lat=%s" % (sys.argv[2], d["value"], d["ms_per_step"], d.get("verdicts_ok"),
      w.get("value"), (d.get("roofline") or {}).get("avg_launch_ms"), d.get("block_latency_ms")))
PY
  return $rc
}
fatal() { [ "$1" -ne 0 ]; }
run base        $B; fatal $? && exit 1
run agg_own     MBLS_AGG_STREAM=own $B; fatal $? && exit 1
run agg_own_pri MBLS_AGG_STREAM=own MBLS_AGG_PRIO=1 $B; fatal $? && exit 1
run base2       $B; fatal $? && exit 1
run lg2         MBLS_LIB_PATH=$PWD/lambda_ethereum_consensus_amd/lib/var_lg2/libmbls.so $B; fatal $? && exit 1
run blk_base    python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline; fatal $? && exit 1
run blk_lg2     MBLS_LIB_PATH=$PWD/lambda_ethereum_consensus_amd/lib/var_lg2/libmbls.so python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline; fatal $? && exit 1
