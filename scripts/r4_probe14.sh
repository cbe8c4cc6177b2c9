#!/bin/bash
# small-batch potrf: left-looking with the fused steps only while they fill the device
set -euo pipefail
mkdir -p gpurun_out/probe14
echo "== default"
PROBE_SHAPES=1000x64,1000x128 timeout -k 10 200 python3 -u scripts/potrf_probe.py 2>&1 | grep batch
for fm in 128 256 384 512; do
  echo "== OB 1024, fuse_min $fm"
  GPMPC_POTRF_OB=1024 GPMPC_POTRF_FUSE_MIN=$fm PROBE_SHAPES=1000x64,1000x128 timeout -k 10 200 \
    python3 -u scripts/potrf_probe.py 2>&1 | grep batch
done
