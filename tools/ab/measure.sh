#!/bin/bash
# One measurement session on the GPU box: the driver's bench line, the rocprofv3 kernel
# statistics of the same command, and separate PMC passes (HBM fetch, HBM write, SQ issue /
# occupancy / LDS counters).  Every GPU step has its own time limit; the chain stops at the
# first failure.  Outputs under gpurun_out/$TAG_*.
#   TAG=r02 BENCH_ARGS="..." tools/measure.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r02}
A="${BENCH_ARGS:-}"
SHORT="--steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-extra-legs $A"
step() { local name=$1; shift; echo "== $name"; "$@" > "gpurun_out/${T}_$name.log" 2>&1; local rc=$?; tail -3 "gpurun_out/${T}_$name.log"; echo "== $name rc=$rc"; return $rc; }
step bench timeout -k 10 600 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} $A &&
step rocprof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline $A &&
if [ "${PMC:-1}" = 1 ]; then
  export MBLS_KEY_CU_RESERVE=0  # rocprofv3 counter collection segfaults at exit with a CU-masked queue (r02)
  step pmc_fetch timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${T}_pmc_fetch -o run --output-format csv -- python bench.py $SHORT &&
  step pmc_write timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${T}_pmc_write -o run --output-format csv -- python bench.py $SHORT &&
  step pmc_sq timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/${T}_pmc_sq -o run --output-format csv -- python bench.py $SHORT &&
  python tools/pmc_traffic.py gpurun_out/${T}_pmc_fetch gpurun_out/${T}_pmc_write gpurun_out/${T}_pmc_traffic.json
fi
