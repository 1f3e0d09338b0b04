#!/bin/bash
# r03: two latency key streams (kstream2) -- parity subset, block latency A/B, warm epoch, timeline
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03g3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests -k "lane_group or mainnet or one_lane or table or multi_engine or deferred or sync_committee" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
try:
    d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]
except Exception as e:
    print(sys.argv[2], "no result", e); sys.exit(0)
w = d.get("warm") or {}
print("%-16s value=%10.1f ms=%7.3f ok=%s warm=%s lat=%s" % (sys.argv[2], d["value"], d["ms_per_step"], d.get("verdicts_ok"), w.get("value"), d.get("block_latency_ms")))
PY
}
for v in 2 1 2 1; do
  MBLS_LAT_KEY_STREAMS=$v timeout -k 10 200 python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline > $OUT/blk$v.json 2> $OUT/blk$v.err || exit 1
  summ $OUT/blk$v.json blk_kstreams$v
done
for v in 2 1; do
  MBLS_LAT_KEY_STREAMS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs > $OUT/ep$v.json 2> $OUT/ep$v.err || exit 1
  summ $OUT/ep$v.json epoch_kstreams$v
done
export TMPDIR=/tmp
R=$(pwd)
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/blkprof -o run -- python3 $R/bench.py --workload mainnet_block --steps 5 --warmup 1 --no-cpu-baseline > $R/$OUT/blkprof.log 2>&1) || exit 1
python3 tools/block_timeline.py $(find $OUT/blkprof -name '*kernel_trace.csv' | head -1) | tail -14
