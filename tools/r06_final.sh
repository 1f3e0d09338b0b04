#!/bin/bash
# r06 closing measurements of the final build, in parts that each fit one gpurun call:
#   PART=a  the -m gpu suite, smoke, PMC traffic passes (FETCH_SIZE / WRITE_SIZE) of the cold
#           epoch and gossip lines
#   PART=b  PMC passes of the deposit and block lines, then every bench line with its same-build
#           traffic (the passes' summaries copied into profiles/ first), and rocprofv3
#           --kernel-trace --stats of the default bench and the secondary workloads
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06final
mkdir -p "$O"
step() { local name=$1; shift; echo "== $name $(date +%T)"; "$@" > "$O/$name.log" 2>&1; local rc=$?; tail -4 "$O/$name.log"; echo "== $name rc=$rc"; return $rc; }
copy_traffic() {  # pass summaries -> the profiles/ names bench.py reads (same build, same knobs)
  for p in "epoch_replay_cold cold_epoch_final" "gossip_verify gossip_final" "deposit_av deposit_final" "mainnet_block block_final"; do
    set -- $p
    [ -f "$O/pmc/$1_traffic.json" ] && cp "$O/pmc/$1_traffic.json" "profiles/r06_pmc_traffic_$2.json" && cp "$O/pmc/$1_traffic.json" "$O/r06_pmc_traffic_$2.json"
  done
  return 0
}
if [ "${PART:-a}" = a ]; then
  step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider &&
  step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" &&
  WORKLOADS="epoch_replay_cold gossip_verify" PASSES="fetch write" OUT=r06final/pmc PASS_LIMIT=200 tools/pmc_passes.sh
else
  WORKLOADS="deposit_av mainnet_block" PASSES="fetch write" OUT=r06final/pmc PASS_LIMIT=200 tools/pmc_passes.sh &&
  copy_traffic &&
  step bench timeout -k 10 600 python bench.py --steps 20 --warmup 5 &&
  for w in gossip_verify deposit_av mainnet_block signing_roots; do
    step "bench_$w" timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 || exit 1
  done &&
  step prof_default timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_default" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs &&
  for w in gossip_verify deposit_av mainnet_block; do
    step "prof_$w" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$w" -o run --output-format csv -- python bench.py --workload $w --steps 20 --warmup 5 || exit 1
  done
fi
