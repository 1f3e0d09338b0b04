#!/bin/bash
# Kernel trace of the default bench line under the given env (ENVS="A=1 B=2"), warm timeline + occupancy.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT:-trace}
mkdir -p $OUT
ROOTD=$(pwd)
cd /tmp && export TMPDIR=/tmp
env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOTD/$OUT/prof -o run -- python3 $ROOTD/bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs --no-roofline > $ROOTD/$OUT/prof.log 2>&1
echo "rocprof rc=$?"
cd $ROOTD
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python3 tools/warm_occupancy.py $f --calls ${STEPS:-20} > $OUT/occupancy.txt; tail -8 $OUT/occupancy.txt
exit 0
