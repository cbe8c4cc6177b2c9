#!/bin/bash
# potrf fused step: C-initialised accumulators, interleaved solve columns, look-ahead
# diagonal update (GPMPC_POTRF_LA): parity, then batch 256 / 1024 timing with LA on / off
set -euo pipefail
mkdir -p gpurun_out/probe7
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "potrf or fit or fitc or exact or trsm or simple3dof or structured or vfe or append or lml or surfaces or fleet_closed or posterior" \
  > gpurun_out/probe7/tests.log 2>&1
echo tests ok
for la in 1 0; do
  GPMPC_POTRF_LA=$la PROBE_SHAPES=1000x256,1000x1024,1000x512,2000x64 timeout -k 10 300 python3 -u scripts/potrf_probe.py \
    > gpurun_out/probe7/potrf_la$la.log 2>&1
done
cat gpurun_out/probe7/potrf_la*.log
timeout -k 10 120 python3 -u scripts/gemm_loop_probe.py > gpurun_out/probe7/gemm_loop.log 2>&1
bash scripts/pmc_mfma.sh gemmloop python3 scripts/gemm_loop_probe.py > /dev/null 2>&1
cat gpurun_out/probe7/gemm_loop.log; head -4 gpurun_out/pmc_mfma_gemmloop/summary.txt
