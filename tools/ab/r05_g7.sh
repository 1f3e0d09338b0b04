set -o pipefail
mkdir -p gpurun_out/r05/g7
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/g7/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05/g7/trace_bench.json 2> gpurun_out/r05/g7/trace_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/g7/trace_dep -o run --output-format csv -- python bench.py --workload deposit_av --steps 20 --warmup 2 > gpurun_out/r05/g7/trace_deposit.json 2> gpurun_out/r05/g7/trace_deposit.err || exit 1
WORKLOADS="epoch_replay_cold deposit_av" PASSES="fetch write sq" OUT=r05/g7/pmc tools/r05_pmc.sh || exit 1
WORKLOADS="epoch_replay_cold" PASSES="insts" PASS_LIMIT=120 OUT=r05/g7/pmc tools/r05_pmc.sh || echo "insts pass failed (counter set not available?)"
echo all-done
