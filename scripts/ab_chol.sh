#!/bin/bash
# A/B of the Cholesky leg (potrf batches, SYRK sets) over library builds:
#   bash scripts/ab_chol.sh "A B" [reps]   (ab/libgpmpc_<name>.so, GPMPC_LIB)
set -euo pipefail
NAMES=$1; REPS=${2:-2}
for r in $(seq 1 "$REPS"); do
  for n in $NAMES; do
    out=$(GPMPC_LIB=ab/libgpmpc_$n.so timeout -k 10 200 python3 scripts/chol_probe.py 2>/dev/null | grep '^{')
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], {b: v['frac_fp64_peak'] for b, v in d['by_batch'].items()}, 'syrk_potrf', d['syrk_potrf']['frac_fp64_peak'], 'syrk_fitc', d['syrk_fitc']['frac_fp64_peak'])" "$n" "$out"
  done
done
