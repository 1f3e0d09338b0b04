#!/bin/bash
# r03 A/B 10: key-grid block size (variant libraries, MBLS_LIB_PATH) on the cold epoch, and the
# aggregate_verify verdict on 6-lane groups vs padded 8-lane groups (deposit AV).
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ab10
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
V=lambda_ethereum_consensus_amd/lib
for cfg in "MBLS_KEY_BLOCK_LIB=default" "MBLS_LIB_PATH=$V/var_kb128/libmbls.so" "MBLS_LIB_PATH=$V/var_kb512/libmbls.so" "MBLS_KEY_BLOCK_LIB=default" "MBLS_LIB_PATH=$V/var_kb128/libmbls.so" "MBLS_LIB_PATH=$V/var_kb512/libmbls.so"; do
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs --no-warm > $OUT/ep.json 2> $OUT/ep.err
  rc=$?; fatal $rc && { tail -3 $OUT/ep.err; exit $rc; }
  python3 -c "import json;d=json.loads(open('$OUT/ep.json').read().splitlines()[0]);print('$cfg'.split('/')[-2] if '/' in '$cfg' else 'default','cold',d['value'],d['verdicts_ok'],d['roofline']['avg_launch_ms'])"
done
for cfg in "MBLS_LG6=1" "MBLS_LG6=0" "MBLS_LG6=1" "MBLS_LG6=0"; do
  env $cfg timeout -k 10 300 python bench.py --workload deposit_av --steps 20 --warmup 3 --no-cpu-baseline > $OUT/av.json 2> $OUT/av.err
  rc=$?; fatal $rc && { tail -3 $OUT/av.err; exit $rc; }
  python3 -c "import json;d=json.loads(open('$OUT/av.json').read().splitlines()[0]);print('$cfg','deposit_av',d['value'],d.get('verdicts_ok'))"
done
exit 0
