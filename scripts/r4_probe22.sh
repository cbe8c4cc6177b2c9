#!/bin/bash
# batched potrf in k chunks on side streams (GPMPC_POTRF_SPLIT=k) vs one stream, then its parity test
set -euo pipefail
mkdir -p gpurun_out/probe22
for k in 0 2 4 0 2; do
  GPMPC_POTRF_SPLIT=$k PROBE_SHAPES=1000x256,1000x512,1000x1024 timeout -k 10 200 python3 -u scripts/potrf_probe.py \
    > gpurun_out/probe22/split$k.log 2>&1
  echo "== split $k"; grep batch gpurun_out/probe22/split$k.log
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 280 --timeout-method thread \
  -k "switch_paths" > gpurun_out/probe22/tests.log 2>&1
tail -1 gpurun_out/probe22/tests.log
