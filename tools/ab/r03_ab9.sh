#!/bin/bash
# r03 A/B 9: the 8-lane verdict on 6-lane groups (mbls_k_lg6.hip) -- parity of the forced forms
# and the table epoch, then warm epoch lg6 vs padded 8-lane, and one mainnet block.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab9
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests -k "lane_group_forms or table or deferred or mainnet or telemetry or aggregate_lane" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "MBLS_LG6=1" "MBLS_LG6=0" "MBLS_LG6=1" "MBLS_LG6=0"; do
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs > $OUT/ep.json 2> $OUT/ep.err
  rc=$?; fatal $rc && { tail -3 $OUT/ep.err; exit $rc; }
  python3 -c "import json;d=json.loads(open('$OUT/ep.json').read().splitlines()[0]);w=d['warm'];print('$cfg','cold',d['value'],d['verdicts_ok'],'warm',w['value'],w['verdicts_ok'])"
done
for cfg in "MBLS_LG6=1" "MBLS_LG6=0"; do
  env $cfg timeout -k 10 200 python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline > $OUT/block.json 2> $OUT/block.err
  rc=$?; fatal $rc && exit $rc
  python3 -c "import json;d=json.loads(open('$OUT/block.json').read().splitlines()[0]);print('$cfg','block',d['value'],d.get('block_latency_ms'))"
done
exit 0
