#!/bin/bash
# r02 final GPU pass: the whole -m gpu suite, smoke, then one bench line per workload
# (gpurun_out/quick_perf.txt + quick_<workload>.log).  Each GPU step has its own limit.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/final_tests.log 2>&1 || { tail -40 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
TESTS="golden" WORKLOADS="${WORKLOADS:-mainnet_block epoch_replay_cold gossip_verify deposit_av signing_roots}" STEPS=20 bash tools/quick_perf.sh
