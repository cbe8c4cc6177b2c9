#!/bin/bash
# A/B of the 6-DoF rollouts leg over alternative builds of the library:
#   bash scripts/ab_lib.sh "A B C" [reps]   (ab/libgpmpc_<name>.so, GPMPC_LIB)
set -euo pipefail
NAMES=$1; REPS=${2:-1}
for r in $(seq 1 "$REPS"); do
  for n in $NAMES; do
    out=$(GPMPC_LIB=ab/libgpmpc_$n.so BATCHES=${BATCHES:-64} timeout -k 10 120 python3 scripts/rollouts6_probe.py 2>/dev/null)
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); k=d['kernels']; print(sys.argv[1], {b: d[b]['ms_per_step'] for b in d if b.isdigit()}, 'predict', k['predict']['ms'], 'control', k['control']['ms'])" "$n" "$out"
  done
done
