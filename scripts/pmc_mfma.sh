#!/bin/bash
# MFMA utilisation and effective clock per kernel (rocprofv3 --pmc, one pass of
# 8 SQ + 1 GRBM counters) for a command, e.g.
#   bash scripts/pmc_mfma.sh TAG python3 scripts/potrf_probe.py
# Output: gpurun_out/pmc_mfma_TAG/ (csv) + summary by scripts/pmc_mfma.py.
set -euo pipefail
TAG=$1; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_mfma_$TAG
mkdir -p "$OUT"
ARGS=()
for a in "$@"; do if [ -e "$a" ]; then ARGS+=("$(realpath "$a")"); else ARGS+=("$a"); fi; done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_LDS \
  --kernel-trace --output-format csv -d "$OUT" -o run -- "${ARGS[@]}" > "$OUT/cmd.log" 2>&1
cd "$ROOT"
python3 scripts/pmc_mfma.py "$(find "$OUT" -name '*counter_collection.csv' | head -1)" \
  "$(find "$OUT" -name '*kernel_trace.csv' | head -1)" > "$OUT/summary.txt"
echo "summary in $OUT/summary.txt"
