#!/bin/bash
# The driver's default bench command N times back to back (each under its own limit; stops at the
# first failure), then the forced-form tests: a check that the default configuration never hits
# the runtime's resource limits.  Output: gpurun_out/$OUT/.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT:-robust}
mkdir -p $OUT
for i in $(seq 1 ${N:-2}); do
  timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench$i.json 2> $OUT/bench$i.err \
    || { echo "bench $i failed"; grep -h -E "OUT_OF_RESOURCES|Error" $OUT/bench$i.err | head -3; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/bench$i.json') if l.startswith('{')][0]); print('run $i cold', d['value'], 'warm', d['warm']['value'], 'ok', d['verdicts_ok'], d['warm']['verdicts_ok'])"
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_forced_forms.py > $OUT/forced.log 2>&1; rc=$?; tail -1 $OUT/forced.log; exit $rc
