#!/bin/bash
# GPU tests + the configs[1] fit probe with its kernel / HIP-API trace (through gpurun)
set -euo pipefail
ROOT=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gputest.log 2>&1
OUT=$ROOT/gpurun_out/fitprobe
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$ROOT/scripts/fit_probe.py" > "$OUT/probe.log" 2>&1
echo done
