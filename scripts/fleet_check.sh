#!/bin/bash
# 3-DoF fleet on the GPU box: the fleet parity tests, a short bench line (no CPU leg)
# and the main workload's kernel trace and PMC traffic passes (scripts/profile_round.sh).
# Usage: bash scripts/fleet_check.sh TAG
set -euo pipefail
TAG=${1:-fleet}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fleet_parity.py -x -v --timeout 300 \
  --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-chol > "$OUT/bench.log" 2>&1
bash scripts/profile_round.sh "$TAG" "trace fetch write" > "$OUT/prof.log" 2>&1
