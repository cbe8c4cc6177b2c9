#!/bin/bash
# Round-end check on the GPU box, part A: the whole GPU suite, then the default bench line.
# Usage: bash scripts/r5_final_a.sh TAG
set -euo pipefail
TAG=${1:-r5final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
GT_TIMEOUT=800 bash scripts/gputest.sh "$TAG"
timeout -k 10 360 python3 bench.py > "$OUT/bench.log" 2>&1
grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"
