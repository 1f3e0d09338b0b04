#!/bin/bash
# r03: telemetry + table/deferred parity after the last engine edit, one default bench line
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03g15
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests -k "telemetry or table or deferred or aggregate_verify or gossip" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().splitlines()[0]);print('cold',d['value'],'warm',d['warm']['value'],'frac',d['roofline']['frac'],'ok',d['verdicts_ok'],d['warm']['verdicts_ok'])"
