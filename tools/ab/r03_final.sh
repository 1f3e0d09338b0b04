#!/bin/bash
# r03 closing GPU pass: the whole -m gpu suite, smoke, the driver's default bench line (20 steps),
# the per-workload lines, and the rocprofv3 kernel statistics of the default bench command.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03final
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests > $OUT/gputest.log 2>&1
rc=$?; tail -2 $OUT/gputest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cut -c1-300 $OUT/bench.json; fatal $rc && exit $rc
for w in gossip_verify mainnet_block deposit_av signing_roots; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err
  rc=$?; fatal $rc && exit $rc
  python3 -c "import json;d=json.loads(open('$OUT/$w.json').read().splitlines()[0]);print('$w',d['value'],d['unit'],d.get('block_latency_ms'))"
done
ROOTD=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTD/$OUT/prof -o run -- python3 $ROOTD/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $ROOTD/$OUT/prof.log 2>&1
echo "rocprof rc=$?"
exit 0
