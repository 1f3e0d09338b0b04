#!/bin/bash
# Kernel trace of the mainnet-block workload (latency path): gpurun_out/blk${TAG}/
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/blk${TAG:-} -o run --output-format csv -- python bench.py --workload mainnet_block --steps 5 --warmup 1 --no-cpu-baseline --no-rlc --no-extra-legs > gpurun_out/blk${TAG:-}.log 2>&1
