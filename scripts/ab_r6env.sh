#!/bin/bash
# A/B of environment settings on the configs[4] rollouts timing (scripts/rollouts6_probe.py):
#   bash scripts/ab_r6env.sh OUTDIR "VAR=a VAR=b ..." [reps]     ("-" = no setting)
set -euo pipefail
OUT=$1; SETS=$2; REPS=${3:-1}
mkdir -p "$OUT"
for r in $(seq 1 "$REPS"); do
  for S in $SETS; do
    if [ "$S" = - ]; then out=$(timeout -k 10 300 python3 scripts/rollouts6_probe.py 2>/dev/null | grep '^{')
    else out=$(env "$S" timeout -k 10 300 python3 scripts/rollouts6_probe.py 2>/dev/null | grep '^{'); fi
    python3 -c "
import json,sys
d=json.loads(sys.argv[2])
print(sys.argv[1], d['64']['ms_per_step'], d['512']['ms_per_step'], d['64']['launched_steps'], d['512']['launched_steps'])" "$S" "$out" | tee -a "$OUT/ab.log"
  done
done
