#!/bin/bash
# 6-DoF rollouts on the GPU box: the configs[4] / GPMPC parity tests, the 64 / 512
# rollout timing (scripts/rollouts6_probe.py) and the 64-rollout kernel trace and
# PMC traffic passes (scripts/profile_round.sh).  Usage: bash scripts/r6_check.sh TAG
set -euo pipefail
TAG=${1:-r6}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollouts6.py tests/test_gpu_gpmpc6.py -x -v --timeout 300 \
  --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
timeout -k 10 300 python scripts/rollouts6_probe.py > "$OUT/probe.json" 2> "$OUT/probe.err"
bash scripts/profile_round.sh "$TAG" "r6trace r6fetch r6write" > "$OUT/prof.log" 2>&1
