#!/bin/bash
# r03 GPU pass 4 (HEAD after the restore): whole -m gpu suite, smoke, a 20-step default bench
# line, and one rocprofv3 kernel trace (csv + stats) of the cold + warm legs for the timelines.
# Each GPU step has its own limit; a fault / abort / timeout (rc other than 0 or 1) ends it.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03g4
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; fatal $rc && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; fatal $rc && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cut -c1-600 $OUT/bench.json; fatal $rc && exit $rc
ROOTD=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTD/$OUT/prof -o run -- python3 $ROOTD/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-rlc --no-extra-legs > $ROOTD/$OUT/prof.log 2>&1
echo "rocprof rc=$?"
tail -3 $ROOTD/$OUT/prof.log
