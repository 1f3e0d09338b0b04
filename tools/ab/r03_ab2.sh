#!/bin/bash
# r03 A/B 2: hardware queues (8 / 10 / 12) with two latency key streams: block latency and
# pipelined rate, warm and cold epoch
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab2
mkdir -p $OUT
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
for q in 8 10 12 8; do
  for k in 2 1; do
    MBLS_HW_QUEUES=$q MBLS_LAT_KEY_STREAMS=$k timeout -k 10 200 python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline > $OUT/blk_q${q}_k$k.json 2> $OUT/blk.err || exit 1
    summ $OUT/blk_q${q}_k$k.json blk_q${q}_k$k
  done
  MBLS_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs > $OUT/ep_q$q.json 2> $OUT/ep.err || exit 1
  summ $OUT/ep_q$q.json epoch_q$q
done
for v in 1 0; do
  MBLS_LG16_PREP=$v timeout -k 10 200 python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline > $OUT/blk_prep16_$v.json 2> $OUT/blk.err || exit 1
  summ $OUT/blk_prep16_$v.json blk_prep16_$v
done
export TMPDIR=/tmp
R=$(pwd)
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/warmprof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-rlc --no-extra-legs > $R/$OUT/warmprof.log 2>&1) || exit 1
echo done
