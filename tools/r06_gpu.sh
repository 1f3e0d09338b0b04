#!/bin/bash
# r06 GPU session: [pytest targets] -> smoke -> bench (default line).  TESTS (default: the whole
# -m gpu suite), BENCH_STEPS (0 = no bench), BENCH_ARGS.  Each GPU step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r06}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1; shift; echo "== $name"; "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -8 "$OUT/$name.log"; echo "== $name rc=$rc"; return $rc; }
step tests timeout -k 10 ${TEST_TIMEOUT:-1000} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider &&
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" &&
if [ "${BENCH_STEPS:-20}" != 0 ]; then
  step bench timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-20} --warmup 5 ${BENCH_ARGS:-}
fi
