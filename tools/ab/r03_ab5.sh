#!/bin/bash
# r03 A/B 5: warm epoch with the one-lane signature decode + H(m) (MBLS_WARM_PREP=onelane) after
# the narrow-group table gather; queue counts; plus a kernel trace of the one-lane-prep warm leg.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab5
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
try:
    d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]
except Exception as e:
    print(sys.argv[2], "no result", e); sys.exit(0)
w = d.get("warm") or {}
print("%-50s value=%9.1f ms=%7.3f ok=%s warm=%s wok=%s" % (sys.argv[2], d["value"], d["ms_per_step"], d.get("verdicts_ok"), w.get("value"), w.get("verdicts_ok")))
PY
}
for cfg in "MBLS_HW_QUEUES=10" "MBLS_WARM_PREP=onelane" "MBLS_WARM_PREP=onelane MBLS_HW_QUEUES=12" "MBLS_WARM_PREP=onelane MBLS_AGG_LANES_IDX=8" "MBLS_WARM_PREP=onelane MBLS_HW_QUEUES=8" "MBLS_HW_QUEUES=10" "MBLS_WARM_PREP=onelane"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs > $OUT/$tag.json 2> $OUT/$tag.err
  rc=$?; fatal $rc && { tail -3 $OUT/$tag.err; exit $rc; }
  summ $OUT/$tag.json "$cfg"
done
ROOTD=$(pwd)
cd /tmp && export TMPDIR=/tmp
MBLS_WARM_PREP=onelane timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOTD/$OUT/prof -o run -- python3 $ROOTD/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-rlc --no-extra-legs > $ROOTD/$OUT/prof.log 2>&1
echo "rocprof rc=$?"
