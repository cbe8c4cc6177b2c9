#!/bin/bash
# A/B of whole libraries on the configs[4] rollouts timing (scripts/rollouts6_probe.py):
#   bash scripts/ab_r6.sh OUTDIR "default ab/libgpmpc_X.so ..." [reps]
# Lines: lib ms_per_step at 64 and 512 rollouts
set -euo pipefail
OUT=$1; LIBS=$2; REPS=${3:-1}
mkdir -p "$OUT"
for r in $(seq 1 "$REPS"); do
  for L in $LIBS; do
    if [ "$L" = default ]; then unset GPMPC_LIB; else export GPMPC_LIB=$L; fi
    out=$(timeout -k 10 300 python3 scripts/rollouts6_probe.py 2>/dev/null | grep '^{')
    python3 -c "
import json,sys
d=json.loads(sys.argv[2])
print(sys.argv[1], d['64']['ms_per_step'], d['512']['ms_per_step'], d['64']['launched_steps'], d['512']['launched_steps'])" "$L" "$out" | tee -a "$OUT/ab.log"
  done
done
