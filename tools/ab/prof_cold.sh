#!/bin/bash
# Kernel timeline of the cold epoch leg (rocprofv3 kernel trace) for pipeline analysis.
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cold -o run --output-format csv -- python bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-rlc --no-extra-legs > gpurun_out/cold.log 2>&1
