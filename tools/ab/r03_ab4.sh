#!/bin/bash
# r03 A/B 4: per-set key sums with narrower lane groups (MBLS_AGG_LANES cold / MBLS_AGG_LANES_IDX
# table): parity tests of the forced forms, then cold + warm epoch per configuration.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab4
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests -k "aggregate_lane_groups or lane_group_forms or one_lane_cold or table or aggregate" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
try:
    d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]
except Exception as e:
    print(sys.argv[2], "no result", e); sys.exit(0)
w = d.get("warm") or {}
print("%-34s value=%9.1f ms=%7.3f ok=%s warm=%s wok=%s" % (sys.argv[2], d["value"], d["ms_per_step"], d.get("verdicts_ok"), w.get("value"), w.get("verdicts_ok")))
PY
}
for cfg in "MBLS_AGG_LANES=64 MBLS_AGG_LANES_IDX=64" "MBLS_AGG_LANES=32 MBLS_AGG_LANES_IDX=16" "MBLS_AGG_LANES=16 MBLS_AGG_LANES_IDX=8" "MBLS_AGG_LANES=32 MBLS_AGG_LANES_IDX=32" "MBLS_AGG_LANES=64 MBLS_AGG_LANES_IDX=64" "MBLS_AGG_LANES=32 MBLS_AGG_LANES_IDX=16"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs > $OUT/$tag.json 2> $OUT/$tag.err
  rc=$?; fatal $rc && { tail -3 $OUT/$tag.err; exit $rc; }
  summ $OUT/$tag.json "$cfg"
done
