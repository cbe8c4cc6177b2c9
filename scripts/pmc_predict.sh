#!/bin/bash
# Memory-pipeline counters of the 6-DoF rollouts leg (64 rollouts), two --pmc
# passes (SQ instruction mix; TA / TD / TCP busy and stall cycles), summed per
# kernel by scripts/pmc_sum.py:  bash scripts/pmc_predict.sh TAG
set -euo pipefail
TAG=${1:-r3}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_pred_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BATCHES=64 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY \
  SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p1" -o run -- \
  python3 "$ROOT/scripts/rollouts6_probe.py" > "$OUT/p1.log" 2>&1
BATCHES=64 timeout -s KILL 240 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum \
  TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/scripts/rollouts6_probe.py" > "$OUT/p2.log" 2>&1
cd "$ROOT"
for p in p1 p2; do
  python3 scripts/pmc_sum.py "$(find "$OUT/$p" -name '*counter_collection.csv' | head -1)" k_r6_ > "$OUT/$p.txt"
done
echo "summaries in $OUT"
