#!/bin/bash
# r03 A/B 3: warm epoch -- one-lane signature decode + H(m) for table calls, key-stream
# alternation for table calls, 8 vs 10 hardware queues
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab3
mkdir -p $OUT
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
try:
    d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]
except Exception as e:
    print(sys.argv[2], "no result", e); sys.exit(0)
w = d.get("warm") or {}
r = (w.get("roofline") or {})
print("%-22s value=%9.1f ok=%s warm=%s wok=%s chip=%s kern=%s" % (sys.argv[2], d["value"], d.get("verdicts_ok"), w.get("value"), w.get("verdicts_ok"), r.get("chip_frac"),
      {k: v.get("avg_launch_ms") for k, v in (r.get("kernels") or {}).items()}))
PY
}
i=0
for cfg in "MBLS_HW_QUEUES=8" "MBLS_HW_QUEUES=8 MBLS_WARM_PREP=onelane" "MBLS_HW_QUEUES=10" "MBLS_HW_QUEUES=10 MBLS_WARM_PREP=onelane" "MBLS_HW_QUEUES=10 MBLS_LAT_KEY_ALT=all" "MBLS_HW_QUEUES=10 MBLS_WARM_PREP=onelane MBLS_LAT_KEY_ALT=all" "MBLS_HW_QUEUES=8" "MBLS_HW_QUEUES=8 MBLS_WARM_PREP=onelane"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs > $OUT/c$i.json 2> $OUT/c$i.err || { tail -3 $OUT/c$i.err; exit 1; }
  summ $OUT/c$i.json "$cfg"
done
