#!/bin/bash
# fused potrf update + panel solve, pooled GP handles, batched triangular-inverse GEMMs:
# parity, then potrf timing (fused on / off) and the configs[1] fit
set -euo pipefail
mkdir -p gpurun_out/probe4
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "potrf or fit or fitc or exact or trsm or simple3dof or structured or vfe or append or lml or surfaces" \
  > gpurun_out/probe4/tests.log 2>&1
for f in 1 0; do
  GPMPC_POTRF_FUSE=$f PROBE_SHAPES=1000x256,1000x1024 timeout -k 10 300 python3 -u scripts/potrf_probe.py \
    > gpurun_out/probe4/potrf_fuse$f.log 2>&1
done
timeout -k 10 300 python3 -c "
import json, bench
from gp_mpc_rocket_landing_amd import _lib
print(json.dumps(bench.simple3dof_gp_bench(_lib.Context(0), cpu=False)))" > gpurun_out/probe4/fit_bench.log 2>&1
echo done
