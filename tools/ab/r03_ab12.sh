#!/bin/bash
# r03 A/B 12: (a) the whole -m gpu suite with the 6-lane prep / key-side Miller / final kernels;
# (b) host end-to-end leg (synchronous 2,048-set host batches take the lane-group chain) and one
# mainnet block, 6-lane vs padded 8-lane; (c) the persistent key grid (MBLS_KEY_PERSIST).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab12
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests > $OUT/gputest.log 2>&1
rc=$?; tail -2 $OUT/gputest.log; [ $rc -ne 0 ] && exit $rc
for cfg in "MBLS_LG6=1" "MBLS_LG6=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-warm > $OUT/e2e.json 2> $OUT/e2e.err
  rc=$?; fatal $rc && { tail -3 $OUT/e2e.err; exit $rc; }
  python3 -c "
import json;d=json.loads(open('$OUT/e2e.json').read().splitlines()[0]);h=d.get('host_e2e') or {}
print('$cfg','cold',d['value'],'host_e2e',{k:(v.get('value') if isinstance(v,dict) else v) for k,v in h.items() if k in ('callers_1','callers_3','callers_4','verdicts_ok')})"
  env $cfg timeout -k 10 200 python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline > $OUT/block.json 2> $OUT/block.err
  rc=$?; fatal $rc && exit $rc
  python3 -c "import json;d=json.loads(open('$OUT/block.json').read().splitlines()[0]);print('$cfg','block',d['value'],d.get('block_latency_ms'))"
done
MBLS_KEY_PERSIST=512 timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests -k "epoch_replay or deferred" > $OUT/persist_tests.log 2>&1
rc=$?; tail -1 $OUT/persist_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "MBLS_KEY_PERSIST=0" "MBLS_KEY_PERSIST=512" "MBLS_KEY_PERSIST=1024" "MBLS_KEY_PERSIST=0" "MBLS_KEY_PERSIST=512"; do
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs --no-warm > $OUT/ep.json 2> $OUT/ep.err
  rc=$?; fatal $rc && { tail -3 $OUT/ep.err; exit $rc; }
  python3 -c "import json;d=json.loads(open('$OUT/ep.json').read().splitlines()[0]);print('$cfg','cold',d['value'],d['verdicts_ok'],d['roofline']['avg_launch_ms'])"
done
exit 0
