#!/bin/bash
# r03: the driver's multi-GPU launch line at world size 1 (torch.distributed.run, gloo barrier,
# max-over-ranks timing) on the one-GPU box
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03g16
mkdir -p $OUT
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/torchrun1.json 2> $OUT/torchrun1.err
rc=$?; echo "torchrun rc=$rc"; cut -c1-400 $OUT/torchrun1.json; tail -3 $OUT/torchrun1.err; exit $rc
