#!/bin/bash
# 8-wave posterior tile (GPMPC_POST_W8): parity, then the 1024-landing step with it on / off
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe6
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "fleet or predict or posterior or surfaces or exact or fitc or vfe or simple3dof" \
  > gpurun_out/probe6/tests.log 2>&1
echo tests ok
for w in 1 0; do
  GPMPC_POST_W8=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/probe6/kt$w -o kt \
    --output-format csv -- python3 -u bench.py --steps 20 --warmup 3 --no-cpu --no-chol \
    > gpurun_out/probe6/bench$w.log 2>&1
  echo bench $w ok
done
PROBE_SHAPES=1000x1024 bash scripts/pmc_mfma.sh postw8 python3 bench.py --steps 5 --warmup 2 --no-cpu --no-chol \
  > gpurun_out/probe6/pmc.txt 2>&1
echo done
