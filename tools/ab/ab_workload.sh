#!/bin/bash
# A/B of env settings on one --workload (WL): RUNS="label|ENV=V,...|steps;..." -> gpurun_out/$OUT/ab.txt
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${OUT:-abw}
mkdir -p $OUT
: > $OUT/ab.txt
IFS=';' read -r -a runs <<< "$RUNS"
for r in "${runs[@]}"; do
  IFS='|' read -r label envs steps <<< "$r"
  e=()
  [ "$envs" != "-" ] && IFS=, read -r -a e <<< "$envs"
  env "${e[@]}" timeout -k 10 300 python bench.py --workload $WL --steps $steps --warmup 3 --no-cpu-baseline \
    > $OUT/$label.json 2> $OUT/$label.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$label failed rc=$rc"; tail -5 $OUT/$label.err; exit $rc; fi
  python3 - "$label" "$OUT/$label.json" >> $OUT/ab.txt <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][0])
print(f"{sys.argv[1]:20s} value={d['value']:12.1f} {d['unit']} ms={d['ms_per_step']:8.3f} ok={d['verdicts_ok']} "
      f"lat={d.get('block_latency_ms')} k={d.get('kernels_avg_ms')}")
PY
  tail -1 $OUT/ab.txt
done
exit 0
