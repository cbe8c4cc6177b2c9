#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out/probe18
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "switch_paths" > gpurun_out/probe18/tests.log 2>&1
tail -5 gpurun_out/probe18/tests.log
