#!/bin/bash
# r03 GPU pass 2 (divstep inversion + split latency chain): the whole -m gpu suite, then one
# bench line per workload at the driver's 20 steps, and the fused-prep latency path for A/B.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03g2
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
try:
    d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]
except Exception as e:
    print(sys.argv[2], "no result", e); sys.exit(0)
w = d.get("warm") or {}
print("%-16s value=%10.1f ms=%7.3f ok=%s warm=%s lat=%s kern=%s" % (sys.argv[2], d["value"], d["ms_per_step"], d.get("verdicts_ok"),
      w.get("value"), d.get("block_latency_ms"), d.get("kernels_avg_ms") or (d.get("roofline") or {}).get("other_kernels_avg_ms")))
PY
}
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/epoch.json 2> $OUT/epoch.err; rc=$?; summ $OUT/epoch.json epoch; [ $rc -ne 0 ] && exit $rc
for w in mainnet_block gossip_verify deposit_av signing_roots; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err; rc=$?; summ $OUT/$w.json $w; [ $rc -ne 0 ] && exit $rc
done
MBLS_LAT_SPLIT=0 timeout -k 10 300 python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline > $OUT/block_fused.json 2> $OUT/block_fused.err; rc=$?; summ $OUT/block_fused.json block_fused
exit 0
