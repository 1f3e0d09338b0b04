#!/bin/bash
# PMC passes: per workload, HBM traffic (FETCH_SIZE, WRITE_SIZE: one
# pass each, folded by tools/pmc_traffic.py), issue / occupancy / LDS (8 SQ + GRBM, tools/pmc_sq.py)
# and a dynamic instruction-class split (SQ_INSTS_*), each pass its own rocprofv3 run with
# --kernel-trace only and its own hard time limit; the chain stops at the first failure.
#   WORKLOADS="epoch_replay_cold deposit_av" PASSES="fetch write sq insts" OUT=r05/pmc tools/pmc_passes.sh
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-r05/pmc}
mkdir -p "$OUT"
declare -A CNT=(
  [fetch]="FETCH_SIZE"
  [write]="WRITE_SIZE"
  [sq]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
  [insts]="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VALU_INT64"
  [stall]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_MISSES GRBM_GUI_ACTIVE"
)
for w in ${WORKLOADS:-epoch_replay_cold deposit_av}; do
  args="--workload $w --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-rlc --no-extra-legs"
  [ -n "$LIBV" ] && export MBLS_LIB_PATH=$LIBV
  for p in ${PASSES:-fetch write sq}; do
    echo "== $w $p $(date +%T)"
    timeout -k 10 -s KILL ${PASS_LIMIT:-240} rocprofv3 --pmc ${CNT[$p]} --kernel-trace -d "$OUT/${w}_$p" -o run \
      --output-format csv -- python bench.py $args > "$OUT/${w}_$p.log" 2>&1 \
      || { echo "== $w $p failed"; tail -5 "$OUT/${w}_$p.log"; exit 1; }
  done
  if [ -d "$OUT/${w}_fetch" ] && [ -d "$OUT/${w}_write" ]; then
    python3 tools/pmc_traffic.py "$OUT/${w}_fetch" "$OUT/${w}_write" "$OUT/${w}_traffic.json" || exit 1
  fi
  for p in sq stall; do
    if [ -d "$OUT/${w}_$p" ]; then
      python3 tools/pmc_sq.py "$OUT/${w}_$p" "$OUT/${w}_$p.json" || exit 1
    fi
  done
done
echo "== done $(date +%T)"
