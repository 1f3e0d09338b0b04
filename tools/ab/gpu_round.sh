#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel trace.  Every GPU step
# has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "== $name"; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -5 "gpurun_out/$name.log"; echo "== $name rc=$rc"; return $rc; }
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider &&
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 1 &&
step rocprof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline &&
if [ "${PMC:-0}" = 1 ]; then
  step pmc_fetch timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-extra-legs &&
  step pmc_write timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-extra-legs &&
  python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_traffic.json
fi
