#!/bin/bash
# kernel traces of the mainnet-block workload, split latency chain vs fused prep
set -o pipefail
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out && export TMPDIR=/tmp
R=$(pwd)
for v in split fused; do
  [ $v = fused ] && export MBLS_LAT_SPLIT=0
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/blk_$v -o run -- python3 $R/bench.py --workload mainnet_block --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/blk_$v.log 2>&1) || exit 1
  f=$(find gpurun_out/blk_$v -name '*kernel_trace.csv' | head -1)
  python3 tools/block_timeline.py $f
done
