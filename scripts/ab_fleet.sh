#!/bin/bash
# A/B of whole libraries on the bench's main workload only (no CPU, no Cholesky legs):
#   bash scripts/ab_fleet.sh OUTDIR "default ab/libgpmpc_X.so ..." [reps]
# Lines: lib value ms_per_step {kernel: ms}
set -euo pipefail
OUT=$1; LIBS=$2; REPS=${3:-1}
mkdir -p "$OUT"
for r in $(seq 1 "$REPS"); do
  for L in $LIBS; do
    if [ "$L" = default ]; then unset GPMPC_LIB; else export GPMPC_LIB=$L; fi
    out=$(timeout -k 10 300 python3 bench.py --no-cpu --no-chol --steps 40 --warmup 5 2>/dev/null | grep '^{')
    python3 -c "
import json,sys
d=json.loads(sys.argv[2]); k=d['kernels']
print(sys.argv[1], d['value'], d['ms_per_step'], {x: v['ms'] for x, v in k.items()})" "$L" "$out" | tee -a "$OUT/ab.log"
  done
done
