#!/bin/bash
# r03 A/B 14: key-stream CU reserve for the latency path (one mainnet block), re-checked with the
# split chain and two latency key streams (r02 tuned it with one).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab14
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
for r in 32 16 48 64 0 32 48; do
  MBLS_KEY_CU_RESERVE=$r timeout -k 10 200 python bench.py --workload mainnet_block --steps 20 --warmup 3 --no-cpu-baseline > $OUT/block.json 2> $OUT/block.err
  rc=$?; fatal $rc && exit $rc
  python3 -c "import json;d=json.loads(open('$OUT/block.json').read().splitlines()[0]);print('reserve $r','block',d['value'],d.get('block_latency_ms'))"
done
exit 0
