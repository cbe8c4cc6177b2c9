#!/bin/bash
# rocprofv3 kernel stats of the batched potrf probe (diag128 / panel GEMM / SYRK)
# Usage (from the repo root, through gpurun): bash scripts/profile_potrf.sh TAG
set -euo pipefail
TAG=${1:-r1}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_potrf_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/scripts/potrf_probe.py" > "$OUT/probe.log" 2>&1
echo "profiles in $OUT"
