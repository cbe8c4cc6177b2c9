#!/bin/bash
# GPU tests on the box (run through gpurun from the repo root); the log goes to
# gpurun_out/TAG/tests.log.  Everything after TAG goes to pytest (-k EXPR, test files);
# no file given = the whole tests/ directory.  GT_TIMEOUT: seconds for the whole run.
#   bash scripts/gputest.sh r5a -k "posterior or comm" tests/test_gpu_fleet_parity.py
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ARGS=("$@")
has_path=0
for a in "${ARGS[@]}"; do [[ "$a" == tests* ]] && has_path=1; done
[ $has_path = 1 ] || ARGS+=(tests)
timeout -k 10 "${GT_TIMEOUT:-900}" python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
  "${ARGS[@]}" > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
