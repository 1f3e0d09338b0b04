#!/bin/bash
# r03 GPU pass 1: the new parity tests (deferred one-lane verdicts, lifetimes, host-batch
# one-lane calls, KATs), the whole -m gpu suite, a 20-step bench, the scratch clamp
# (MBLS_SCRATCH_STREAMS=7) and the exit under rocprofv3.  Each GPU step has its own limit;
# a fault / abort / timeout (rc other than 0 or 1) ends the script.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
T="python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_deferred.py tests/test_gpu_kat.py "tests/test_gpu_parity.py::test_one_lane_cold_fav_path" "tests/test_gpu_parity.py::test_lane_group_forms" > $OUT/new_tests.log 2>&1
rc=$?; tail -3 $OUT/new_tests.log; fatal $rc && exit $rc
timeout -k 10 600 $T -m gpu tests > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; fatal $rc && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json | cut -c1-400; fatal $rc && exit $rc
MBLS_SCRATCH_STREAMS=7 timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-warm --no-rlc --no-extra-legs > $OUT/scratch7.json 2> $OUT/scratch7.err
rc=$?; echo "scratch7 rc=$rc"; cut -c1-300 $OUT/scratch7.json; grep -i clamp $OUT/scratch7.err; fatal $rc && exit $rc
ROOTD=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOTD/$OUT/prof -o run -- python3 $ROOTD/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $ROOTD/$OUT/prof.log 2>&1
echo "rocprof rc=$?"
tail -5 $ROOTD/$OUT/prof.log
