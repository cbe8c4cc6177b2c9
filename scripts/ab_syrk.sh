#!/bin/bash
# bash scripts/ab_syrk.sh "A B" [reps]: the FITC SYRK probe over library builds (GPMPC_LIB)
set -euo pipefail
for r in $(seq 1 "${2:-3}"); do for n in $1; do
  echo "$n $(GPMPC_LIB=ab/libgpmpc_$n.so timeout -k 10 120 python3 scripts/syrk_probe.py 2>/dev/null | grep '^{')"
done; done
