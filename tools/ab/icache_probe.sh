#!/bin/bash
# Key-kernel code-size probe: the key kernel alone and inside the cold epoch pipeline, with the
# Fp multiply inlined (default build) vs out of line (lib/var_g1ol: the g1 TU built with
# MBLS_FP_OUTLINE=1), plus the available SQC instruction-cache counters.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/list_avail.txt 2>&1 || echo "list-avail rc=$?"
grep -io "SQC_[A-Z_]*" gpurun_out/list_avail.txt | sort -u | tr '\n' ' '; echo
for v in default g1ol; do
  lib=lambda_ethereum_consensus_amd/lib/libmbls.so
  [ $v != default ] && lib=lambda_ethereum_consensus_amd/lib/var_$v/libmbls.so
  echo "== $v standalone"; MBLS_LIB_PATH=$lib timeout -k 10 120 python tools/diag_keykernel.py 10 || exit 1
done
SETTINGS="- MBLS_LIB_PATH=lambda_ethereum_consensus_amd/lib/var_g1ol/libmbls.so" bash tools/ab_env.sh
