set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH_STEPS=100 PMC=1 bash tools/gpu_round.sh || exit 1
WORKLOADS="gossip_verify" bash tools/profile_workloads.sh || exit 1
timeout -k 10 300 python bench.py --workload gossip_verify > gpurun_out/bench_gossip.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_gossip.log | head -c 600
