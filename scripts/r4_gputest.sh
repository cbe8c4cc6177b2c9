#!/bin/bash
# the GPU test suite (through gpurun); log under gpurun_out/.  PYTEST_K: a -k expression.
set -euo pipefail
mkdir -p gpurun_out
K=()
if [ -n "${PYTEST_K:-}" ]; then K=(-k "$PYTEST_K"); fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${K[@]}" \
  > gpurun_out/gputest.log 2>&1
tail -3 gpurun_out/gputest.log
