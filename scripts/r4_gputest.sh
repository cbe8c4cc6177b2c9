#!/bin/bash
# the GPU test suite (through gpurun); log under gpurun_out/
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/gputest.log 2>&1
tail -3 gpurun_out/gputest.log
