#!/bin/bash
# Closing measurements of a round: the default bench line (the driver's command), the same command
# under rocprofv3 --kernel-trace --stats (the summary the roofline's kernel time must agree with),
# and each extra workload's line under rocprofv3.  Every GPU step has its own time limit; the chain
# stops at the first failure.  Output: gpurun_out/$OUT/.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT:-final}
mkdir -p $OUT
ROOTD=$(pwd)
export TMPDIR=/tmp
STEPS=${STEPS:-20}
if [ -z "$SKIP_DEFAULT" ]; then
  timeout -k 10 420 python bench.py --steps $STEPS --warmup 5 > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
  grep '^{' $OUT/bench.json | head -c 600; echo
  (cd /tmp && timeout -k 10 480 rocprofv3 --kernel-trace --stats -d $ROOTD/$OUT/prof_default -o run --output-format csv -- \
    python3 $ROOTD/bench.py --steps $STEPS --warmup 5 > $ROOTD/$OUT/prof_default.log 2>&1) \
    || { echo "rocprof default failed"; tail -5 $OUT/prof_default.log; exit 1; }
fi
for w in ${WORKLOADS:-gossip_verify mainnet_block deposit_av signing_roots}; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOTD/$OUT/prof_$w -o run --output-format csv -- \
    python3 $ROOTD/bench.py --workload $w --steps $STEPS --warmup 2 > $ROOTD/$OUT/prof_$w.log 2>&1) \
    || { echo "== $w failed"; tail -5 $OUT/prof_$w.log; exit 1; }
  grep '^{' $OUT/prof_$w.log | head -c 300; echo
done
