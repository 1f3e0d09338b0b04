#!/bin/bash
# HBM traffic per kernel launch for every bench workload: two rocprofv3
# --pmc passes per workload (FETCH_SIZE, WRITE_SIZE: one TCC counter group each, --kernel-trace
# only, no other trace domains), folded by tools/pmc_traffic.py into
# gpurun_out/pmc_<workload>.json.  Each pass under its own time limit; the chain stops at the
# first failure.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WORKLOADS:-epoch_replay_cold mainnet_block gossip_verify deposit_av}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== $w $c"
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d "gpurun_out/pmc_${w}_$c" -o run \
      --output-format csv -- python bench.py --workload "$w" --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline \
      --no-rlc --no-extra-legs > "gpurun_out/pmc_${w}_$c.log" 2>&1 \
      || { echo "== $w $c failed"; tail -5 "gpurun_out/pmc_${w}_$c.log"; exit 1; }
  done
  python3 tools/pmc_traffic.py "gpurun_out/pmc_${w}_FETCH_SIZE" "gpurun_out/pmc_${w}_WRITE_SIZE" \
    "gpurun_out/pmc_$w.json" || exit 1
done
