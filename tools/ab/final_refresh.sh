#!/bin/bash
# End-of-round refresh: parity tests, smoke, the default bench line + rocprofv3 kernel stats +
# PMC traffic, then one bench line and kernel-stats summary per secondary workload.
set -o pipefail
cd "$(dirname "$0")/.."
BENCH_STEPS=100 PMC=1 bash tools/gpu_round.sh || exit 1
WORKLOADS="gossip_verify mainnet_block deposit_av" bash tools/profile_workloads.sh || exit 1
for w in gossip_verify mainnet_block deposit_av; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/bench_$w.log 2>&1 || exit 1
  grep '^{' gpurun_out/bench_$w.log | head -c 300; echo
done
