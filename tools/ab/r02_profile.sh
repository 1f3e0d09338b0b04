#!/bin/bash
# r02 closing measurement: the default bench line (all legs, the driver's 20 steps), then the
# rocprofv3 kernel-trace statistics of the same command (the CU-masked latency stream makes
# rocprofv3 segfault at process exit after its CSVs are written, so that step's status is
# judged by the statistics file).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 1 > gpurun_out/final_bench.log 2>&1 || { tail -20 gpurun_out/final_bench.log; exit 1; }
grep '^{' gpurun_out/final_bench.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/final_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 1 --no-cpu-baseline > gpurun_out/final_prof.log 2>&1
rc=$?
echo "rocprof rc=$rc"
test -s gpurun_out/final_prof/run_kernel_stats.csv && head -12 gpurun_out/final_prof/run_kernel_stats.csv | cut -c1-120
