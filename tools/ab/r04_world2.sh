#!/bin/bash
# World-2 rehearsal of the rank path on a one-GPU box: the driver's torchrun line
# with both ranks pinned to cuda:0 (MBLS_BENCH_DEVICE=0), the communicator deadline shortened so a
# refused or hung RCCL set-up ends as a recorded error, not a hang.  Records rc, the JSON line and
# the sharded-table leg's outcome under gpurun_out/$OUT.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUT:-world2}
mkdir -p $OUT
MBLS_BENCH_DEVICE=0 MBLS_COMM_TIMEOUT_MS=${MBLS_COMM_TIMEOUT_MS:-30000} \
  timeout -k 10 ${LIMIT:-420} python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port ${PORT:-29561} bench.py --gpus 2 --steps ${STEPS:-10} --warmup 3 \
  --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "rc=$rc" > $OUT/rc.txt
python3 - "$OUT" "$rc" <<'PY'
import json, sys
out, rc = sys.argv[1], sys.argv[2]
lines = [l for l in open(f"{out}/bench.json") if l.startswith("{")]
rec = {"rc": int(rc), "json_lines": len(lines)}
if lines:
    d = json.loads(lines[-1])
    rec.update(value=d.get("value"), n_gpus=d.get("n_gpus"), verdicts_ok=d.get("verdicts_ok"),
               warm=(d.get("warm") or {}).get("value"), sharded=d.get("warm_sharded_table"))
rec["stderr_tail"] = open(f"{out}/bench.err").read()[-1500:]
print(json.dumps(rec, indent=1))
json.dump(rec, open(f"{out}/summary.json", "w"), indent=1)
PY
exit $rc
