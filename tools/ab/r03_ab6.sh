#!/bin/bash
# r03 A/B 6: fused one-lane G2 prep (mbls_k_g2_prep_1l: signature decode + H(m) in one launch) --
# the whole -m gpu suite with the one-lane warm prep forced, then cold + warm epoch per config,
# and the gossip workload (dev_verify now uses the fused prep too).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab6
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
MBLS_WARM_PREP=onelane timeout -k 10 700 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -ne 0 ] && exit $rc
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
for cfg in "MBLS_HW_QUEUES=10" "MBLS_WARM_PREP=onelane" "MBLS_WARM_PREP=onelane MBLS_HW_QUEUES=12" "MBLS_HW_QUEUES=12" "MBLS_WARM_PREP=onelane MBLS_LG16=1" "MBLS_AGG_STREAM=own" "MBLS_AGG_STREAM=own MBLS_WARM_PREP=onelane MBLS_HW_QUEUES=12" "MBLS_WARM_PREP=onelane MBLS_HW_QUEUES=14" "MBLS_HW_QUEUES=10" "MBLS_WARM_PREP=onelane MBLS_HW_QUEUES=12"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs > $OUT/$tag.json 2> $OUT/$tag.err
  rc=$?; fatal $rc && { tail -3 $OUT/$tag.err; exit $rc; }
  summ $OUT/$tag.json "$cfg"
done
timeout -k 10 200 python bench.py --workload gossip_verify --steps 20 --warmup 3 --no-cpu-baseline > $OUT/gossip.json 2> $OUT/gossip.err
rc=$?; cut -c1-300 $OUT/gossip.json; fatal $rc && exit $rc
timeout -k 10 200 python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline > $OUT/block.json 2> $OUT/block.err
rc=$?; cut -c1-300 $OUT/block.json; fatal $rc && exit $rc
