set -o pipefail
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/blk -o run --output-format csv -- python bench.py --workload mainnet_block --steps 5 --warmup 1 --no-cpu-baseline --no-rlc --no-extra-legs > gpurun_out/blk.log 2>&1
