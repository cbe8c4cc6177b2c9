#!/bin/bash
# potrf: parity at multiple-of-8 batches, XCD-batched row blocks on / off; the configs[4] QP-settings sweep
set -euo pipefail
mkdir -p gpurun_out/probe2
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "potrf_batched_dev" \
  > gpurun_out/probe2/potrf_tests.log 2>&1
for x in 1 0; do
  GPMPC_ROWBLOCK_XCD=$x PROBE_SHAPES=1000x64,1000x256,1000x1024 timeout -k 10 300 python3 -u scripts/potrf_probe.py \
    > gpurun_out/probe2/potrf_xcd$x.log 2>&1
done
timeout -k 10 600 python3 -u scripts/r6_qp_sweep.py > gpurun_out/probe2/r6_sweep.log 2>&1
echo done
