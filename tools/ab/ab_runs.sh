#!/bin/bash
# Generic A/B driver: RUNS is a ';'-separated list of "label|ENV=V,ENV2=V2|steps" (env "-" = none);
# each runs bench.py's default line (cold + warm legs) and prints one summary line to
# gpurun_out/$OUT/ab.txt.  Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${OUT:-ab}
mkdir -p $OUT
: > $OUT/ab.txt
IFS=';' read -r -a runs <<< "$RUNS"
for r in "${runs[@]}"; do
  IFS='|' read -r label envs steps <<< "$r"
  e=()
  [ "$envs" != "-" ] && IFS=, read -r -a e <<< "$envs"
  env "${e[@]}" timeout -k 10 300 python bench.py --steps $steps --warmup 5 --no-cpu-baseline --no-rlc --no-extra-legs \
    ${BENCH_ARGS:-} > $OUT/$label.json 2> $OUT/$label.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$label failed rc=$rc"; tail -5 $OUT/$label.err; exit $rc; fi
  python3 - "$label" "$steps" "$OUT/$label.json" >> $OUT/ab.txt <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][0])
w = d.get("warm") or {}
r = d.get("roofline") or {}
print(f"{sys.argv[1]:24s} steps={sys.argv[2]:>4s} cold={d['value']:9.1f} ms={d['ms_per_step']:7.3f} key_ms={r.get('avg_launch_ms')} "
      f"ok={d['verdicts_ok']} warm={w.get('value')} wms={w.get('ms_per_step')} wok={w.get('verdicts_ok')} "
      f"wk={ {k: v.get('avg_launch_ms') for k, v in ((w.get('roofline') or {}).get('kernels') or {}).items()} }")
PY
  tail -1 $OUT/ab.txt
done
exit 0
