#!/bin/bash
# rocprofv3 kernel-trace summaries of every bench workload (one GPU session; each step under
# its own time limit, the chain stops at the first failure).  Summaries land in
# gpurun_out/prof_<workload>/run_kernel_stats.csv; copy the ones to keep into profiles/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WORKLOADS:-epoch_replay_cold gossip_verify mainnet_block deposit_av signing_roots}; do
  echo "== $w"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$w" -o run --output-format csv -- \
    python bench.py --workload "$w" --steps 10 --warmup 1 --no-cpu-baseline --no-rlc --no-extra-legs \
    > "gpurun_out/prof_$w.log" 2>&1 || { echo "== $w failed"; tail -5 "gpurun_out/prof_$w.log"; exit 1; }
  grep '^{' "gpurun_out/prof_$w.log" | head -c 300; echo
done
