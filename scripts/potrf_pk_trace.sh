#!/bin/bash
# Kernel traces of the batch-1024 potrf probe with the packed-layout diagonal kernel on
# (default) and off: bash scripts/potrf_pk_trace.sh TAG
set -euo pipefail
TAG=${1:-pk}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for pk in 1 0; do
  GPMPC_DIAG_PK=$pk PROBE_SHAPES=1000x1024 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/pk$pk" -o run -- python3 "$ROOT/scripts/potrf_probe.py" > "$OUT/pk$pk.log" 2>&1
done
