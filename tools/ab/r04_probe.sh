#!/bin/bash
# r04 probe: cold + warm legs at the driver's 20 steps and at 100 steps (steady-state period vs
# the pipeline's fill/drain), then a kernel trace of the 20-step line for the warm timeline.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r04probe
mkdir -p $OUT
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
for s in 20 100 20; do
  timeout -k 10 300 python bench.py --steps $s --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs > $OUT/b$s.json 2> $OUT/b$s.err
  rc=$?; fatal $rc && exit $rc
  python3 -c "import json;d=json.loads(open('$OUT/b$s.json').read().splitlines()[0]);w=d['warm'];print('steps $s cold',d['value'],d['ms_per_step'],'warm',w['value'],w['ms_per_step'],w['verdicts_ok'])"
done
ROOTD=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOTD/$OUT/prof -o run -- python3 $ROOTD/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs --no-roofline > $ROOTD/$OUT/prof.log 2>&1
echo "rocprof rc=$?"
cd $ROOTD
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
[ -n "$f" ] && python3 tools/warm_timeline.py $f > $OUT/warm_timeline.txt && tail -8 $OUT/warm_timeline.txt
exit 0
