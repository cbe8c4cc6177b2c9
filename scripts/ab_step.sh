#!/bin/bash
# A/B of the control step under an environment switch: bash scripts/ab_step.sh VAR "v0 v1 ..." [reps]
set -euo pipefail
VAR=$1; VALS=$2; REPS=${3:-2}
for r in $(seq 1 "$REPS"); do
  for v in $VALS; do
    echo -n "$VAR=$v: "
    env "$VAR=$v" timeout -k 10 120 python3 scripts/step_probe.py
  done
done
