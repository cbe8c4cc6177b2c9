#!/bin/bash
# A/B of the bench's main workload under an environment switch (one library):
#   bash scripts/ab_env.sh VAR "v0 v1 ..." [reps]
set -euo pipefail
VAR=$1; VALS=$2; REPS=${3:-2}
for r in $(seq 1 "$REPS"); do
  for v in $VALS; do
    out=$(env "$VAR=$v" timeout -k 10 200 python3 bench.py --no-cpu --no-chol --steps 20 2>/dev/null | grep '^{')
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); k=d['kernels']; print(sys.argv[1], d['value'], d['ms_per_step'], {x: (v['ms'], round(v['frac'], 4)) for x, v in k.items()})" "$VAR=$v" "$out"
  done
done
