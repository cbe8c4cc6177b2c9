#!/bin/bash
# A/B of the bench's main workload over alternative library builds:
#   bash scripts/ab_bench.sh "A B" [reps]   (ab/libgpmpc_<name>.so, GPMPC_LIB)
set -euo pipefail
NAMES=$1; REPS=${2:-2}
for r in $(seq 1 "$REPS"); do
  for n in $NAMES; do
    out=$(GPMPC_LIB=ab/libgpmpc_$n.so timeout -k 10 200 python3 bench.py --no-cpu --no-chol --steps 20 2>/dev/null | grep '^{')
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); k=d['kernels']; print(sys.argv[1], d['value'], d['ms_per_step'], {x: (v['ms'], round(v['frac'], 4)) for x, v in k.items()})" "$n" "$out"
  done
done
