#!/bin/bash
# left-looking potrf from batch 128 (fused from 1 workgroup below 256): parity, then the
# fuse threshold at 256 / 512 / 1024 (512 default vs 1)
set -euo pipefail
mkdir -p gpurun_out/probe12
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "potrf or lml or fit or exact" > gpurun_out/probe12/tests.log 2>&1
tail -1 gpurun_out/probe12/tests.log
PROBE_SHAPES=1000x64,1000x128,1000x192,1000x256,1000x512,1000x1024 timeout -k 10 300 python3 -u scripts/potrf_probe.py \
  > gpurun_out/probe12/potrf_default.log 2>&1
GPMPC_POTRF_FUSE_MIN=1 PROBE_SHAPES=1000x256,1000x512,1000x1024 timeout -k 10 300 python3 -u scripts/potrf_probe.py \
  > gpurun_out/probe12/potrf_fmin1.log 2>&1
grep -h batch gpurun_out/probe12/potrf_default.log gpurun_out/probe12/potrf_fmin1.log
