#!/bin/bash
# The -m gpu suite (or a -k subset: K=...) on the box, log under gpurun_out/$OUT.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT:-gputest}
mkdir -p $OUT
timeout -k 10 ${LIMIT:-900} python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu tests ${K:+-k "$K"} > $OUT/gputest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" $OUT/gputest.log | tail -80 | cut -c1-160
tail -3 $OUT/gputest.log
exit $rc
