#!/bin/bash
# Batched potrf on the GPU box: the potrf parity tests, then the probe at n = 1000 for
# batches 256 / 512 / 1024 with the packed-layout diagonal kernel off and on.
# Usage: bash scripts/potrf_check.sh TAG
set -euo pipefail
TAG=${1:-potrf}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "potrf" -x -v --timeout 300 \
  --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
for pk in 0 1 0 1; do
  GPMPC_DIAG_PK=$pk PROBE_SHAPES=1000x256,1000x512,1000x1024 timeout -k 10 300 python scripts/potrf_probe.py \
    2>&1 | sed "s/^/pk=$pk /" >> "$OUT/probe.log"
done
