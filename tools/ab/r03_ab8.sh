#!/bin/bash
# r03 A/B 8: warm calls rotating over kstream2 too (8 G2 streams): table tests, then 3 epoch runs
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab8
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests -k "table" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs > $OUT/ep$i.json 2> $OUT/ep$i.err
  rc=$?; fatal $rc && { tail -3 $OUT/ep$i.err; exit $rc; }
  python3 -c "import json,sys;d=json.loads(open('$OUT/ep$i.json').read().splitlines()[0]);w=d['warm'];print('cold',d['value'],d['verdicts_ok'],'warm',w['value'],w['verdicts_ok'])"
done
timeout -k 10 200 python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline > $OUT/block.json 2> $OUT/block.err
rc=$?; python3 -c "import json;d=json.loads(open('$OUT/block.json').read().splitlines()[0]);print('block',d['value'],d.get('block_latency_ms'))"; fatal $rc && exit $rc
exit 0
