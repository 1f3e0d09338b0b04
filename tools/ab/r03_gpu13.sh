#!/bin/bash
# r03: forced lane-group forms after making the 6-lane chain opt-in, plus one mainnet block
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03g13
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests -k "lane_group_forms or mainnet or table_epoch or one_lane" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline > $OUT/block.json 2> $OUT/block.err || exit 1
python3 -c "import json;d=json.loads(open('$OUT/block.json').read().splitlines()[0]);print('block',d['value'],d.get('block_latency_ms'))"
