#!/bin/bash
# r03 PMC passes (one counter group per rocprofv3 run, --kernel-trace only): HBM fetch / write of
# the epoch legs (cold + warm, 2 steps) and of one mainnet block, and the SQ issue counters of
# the epoch legs.  Folded by tools/pmc_traffic.py / tools/pmc_sq.py.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03pmc2
mkdir -p $OUT
ROOTD=$(pwd)
export TMPDIR=/tmp MBLS_KEY_CU_RESERVE=0  # counter collection + a CU-masked queue crashed at exit (r02)
EP="--steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-extra-legs --no-rlc"
BL="--workload mainnet_block --steps 2 --warmup 1 --no-cpu-baseline"
run() {  # name counters... -- bench args
  local name=$1; shift
  local ctr=$1; shift
  (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -d $ROOTD/$OUT/$name -o run --output-format csv -- python3 $ROOTD/bench.py "$@") > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
echo "pmc pass 2"
run ep_fetch FETCH_SIZE $EP && run ep_write WRITE_SIZE $EP && run bl_fetch FETCH_SIZE $BL && run bl_write WRITE_SIZE $BL || exit 1
python3 tools/pmc_traffic.py $OUT/ep_fetch $OUT/ep_write $OUT/traffic_epoch.json > /dev/null && python3 tools/pmc_traffic.py $OUT/bl_fetch $OUT/bl_write $OUT/traffic_block.json > /dev/null
(cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $ROOTD/$OUT/ep_sq -o run --output-format csv -- python3 $ROOTD/bench.py $EP) > $OUT/ep_sq.log 2>&1
echo "ep_sq rc=$?"
