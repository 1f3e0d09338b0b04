#!/bin/bash
# Full default bench line (all legs) for the in-tree build and a variant library, alternating.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in ${VARIANTS:-default old}; do
  lib=lambda_ethereum_consensus_amd/lib/libmbls.so
  [ $v != default ] && lib=lambda_ethereum_consensus_amd/lib/var_$v/libmbls.so
  MBLS_LIB_PATH=$lib timeout -k 10 300 python bench.py ${BENCH_ARGS:-} --no-cpu-baseline > gpurun_out/full_$v.log 2>&1 || { tail -5 gpurun_out/full_$v.log; exit 1; }
  python -c "
import json,sys
d=[json.loads(l) for l in open('gpurun_out/full_$v.log') if l.startswith('{')][0]
print('$v', 'cold', d['value'], 'warm', d['warm']['value'], 'warm_rlc', d['warm']['rlc']['value'], 'mixed', d['mixed']['value'], 'host_e2e', d['host_e2e']['value'], 'rlc', d['rlc']['value'])"
done
