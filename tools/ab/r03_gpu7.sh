#!/bin/bash
# r03 GPU pass 7: one-lane warm prep default (n_sets > 1024) -- the epoch-size table parity test,
# the table / aggregate tests, a default 20-step bench line, and a warm-leg kernel trace.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03g7
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests -k "table or aggregate or deferred or epoch" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cut -c1-400 $OUT/bench.json; fatal $rc && exit $rc
ROOTD=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTD/$OUT/prof -o run -- python3 $ROOTD/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-rlc --no-extra-legs > $ROOTD/$OUT/prof.log 2>&1
echo "rocprof rc=$?"
