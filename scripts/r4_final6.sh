#!/bin/bash
# round-4 check: the whole GPU suite, smoke(), then the default bench line
set -euo pipefail
mkdir -p gpurun_out/final6
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/final6/gputest.log 2>&1
tail -2 gpurun_out/final6/gputest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final6/smoke.log 2>&1
timeout -k 10 600 python3 -u bench.py > gpurun_out/final6/bench.log 2>&1
tail -c 600 gpurun_out/final6/bench.log
