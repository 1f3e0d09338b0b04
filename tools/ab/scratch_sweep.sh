#!/bin/bash
# VERDICT r01 #3 check: the cold epoch step at MBLS_SCRATCH_STREAMS = 3..7 (one bench line each,
# a scratch-heavy configuration either aborts or collapses), then the HBM traffic of the
# scratch-carrying kernels (FETCH_SIZE / WRITE_SIZE passes) on the cold epoch and on one
# mainnet block.  Outputs under gpurun_out/${TAG}_*.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r02s}
out=gpurun_out/${T}_sweep.txt
: > "$out"
for s in ${STREAMS:-3 4 5 6 7}; do
  MBLS_SCRATCH_STREAMS=$s timeout -k 10 300 python bench.py --workload epoch_replay_cold --steps 20 --warmup 2 \
    --no-cpu-baseline --no-rlc --no-warm --no-extra-legs > gpurun_out/${T}_s$s.log 2>&1
  rc=$?
  echo "streams=$s rc=$rc $(grep -h '^{' gpurun_out/${T}_s$s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print("value=%.1f ms=%.3f ok=%s" % (d["value"], d["ms_per_step"], d.get("verdicts_ok")))' 2>/dev/null)" | tee -a "$out"
  [ $rc -eq 0 ] || exit 1
done
[ "${PMC:-1}" = 1 ] || exit 0
SHORT="--steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-extra-legs --no-rlc"
export MBLS_KEY_CU_RESERVE=0  # rocprofv3 counter collection segfaults at exit with a CU-masked queue (r02)
for w in epoch_replay_cold mainnet_block; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/${T}_${w}_$c -o run --output-format csv -- \
      python bench.py --workload $w $SHORT > gpurun_out/${T}_${w}_$c.log 2>&1 || { tail -5 gpurun_out/${T}_${w}_$c.log; exit 1; }
  done
  python3 tools/pmc_traffic.py gpurun_out/${T}_${w}_FETCH_SIZE gpurun_out/${T}_${w}_WRITE_SIZE gpurun_out/${T}_${w}_traffic.json
done
