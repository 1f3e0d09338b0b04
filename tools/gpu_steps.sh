#!/bin/bash
# GPU round trip: the -m gpu suite (or a -k subset), then bench lines, each step under its own
# time limit, the chain stopping at the first failure.  Usage (on the box, via gpurun):
#   STEPS="tests bench deposit fill4 fp64 world2" OUT=r05/x tools/gpu_steps.sh
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-r05/run}
mkdir -p "$OUT"
for s in ${STEPS:-tests bench}; do
  echo "== $s $(date +%T)"
  case $s in
    tests)
      timeout -k 10 ${LIMIT:-900} python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider \
        -m gpu tests ${K:+-k "$K"} > "$OUT/gputest.log" 2>&1
      rc=$?
      grep -E "PASSED|FAILED|ERROR|SKIPPED" "$OUT/gputest.log" | tail -100 | cut -c1-150
      tail -3 "$OUT/gputest.log"
      [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
      cat "$OUT/bench.json" | cut -c1-600 ;;
    deposit)
      timeout -k 10 300 python -u bench.py --workload deposit_av --steps 20 --warmup 2 > "$OUT/deposit.json" \
        2> "$OUT/deposit.err" || exit 1
      cat "$OUT/deposit.json" ;;
    deposit1l)
      MBLS_AV_FORM=1l timeout -k 10 300 python -u bench.py --workload deposit_av --steps 20 --warmup 2 \
        > "$OUT/deposit1l.json" 2> "$OUT/deposit1l.err" || exit 1
      cat "$OUT/deposit1l.json" ;;
    gossip|mainnet_block|signing_roots)
      w=$s; [ $s = gossip ] && w=gossip_verify
      timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 2 > "$OUT/$s.json" 2> "$OUT/$s.err" || exit 1
      cat "$OUT/$s.json" | cut -c1-600 ;;
    fill4)  # the r04 abort recipe: MBLS_WARM_FILL=4 through the whole default bench process
      MBLS_WARM_FILL=4 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        > "$OUT/fill4.json" 2> "$OUT/fill4.err" || { tail -20 "$OUT/fill4.err"; exit 1; }
      cat "$OUT/fill4.json" | cut -c1-400 ;;
    fp64)
      timeout -k 10 60 tools/fp_rates_radix28 > "$OUT/fp_rates_radix28.json" || exit 1
      timeout -k 10 60 tools/fp64_mont > "$OUT/fp64_mont.json" || exit 1
      timeout -k 10 60 tools/fp64_mont_w2 >> "$OUT/fp64_mont.json" || exit 1
      cat "$OUT/fp_rates_radix28.json" "$OUT/fp64_mont.json" ;;
    world2)  # the driver's N > 1 launch line, both ranks on this box's one GPU (a rehearsal)
      MBLS_BENCH_DEVICE=0 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline \
        > "$OUT/world2.json" 2> "$OUT/world2.err" || { tail -20 "$OUT/world2.err"; exit 1; }
      cat "$OUT/world2.json" | cut -c1-800 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
