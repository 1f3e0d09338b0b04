#!/bin/bash
# r03 A/B 11: persistent key grid (MBLS_KEY_PERSIST=<blocks>, 64-key chunks from an atomic
# counter) vs the default grid on the cold epoch; parity of the persistent form first.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab11
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
MBLS_KEY_PERSIST=512 timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests -k "epoch_replay or deferred" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "MBLS_KEY_PERSIST=0" "MBLS_KEY_PERSIST=512" "MBLS_KEY_PERSIST=480" "MBLS_KEY_PERSIST=0" "MBLS_KEY_PERSIST=512" "MBLS_KEY_PERSIST=1024"; do
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs --no-warm > $OUT/ep.json 2> $OUT/ep.err
  rc=$?; fatal $rc && { tail -3 $OUT/ep.err; exit $rc; }
  python3 -c "import json;d=json.loads(open('$OUT/ep.json').read().splitlines()[0]);print('$cfg','cold',d['value'],d['verdicts_ok'],d['roofline']['avg_launch_ms'])"
done
exit 0
