#!/bin/bash
# A/B of whole libraries on the bench (main workload + Cholesky/SYRK legs) and the dense
# 128-tile loop probe: bash scripts/ab_libs.sh OUTDIR "default ab/libgpmpc_X.so ..." [reps]
# ("default" = the in-tree library).  Lines: lib value ms_per_step {kernel: (ms, frac)} chol
set -euo pipefail
OUT=$1; LIBS=$2; REPS=${3:-1}
mkdir -p "$OUT"
for r in $(seq 1 "$REPS"); do
  for L in $LIBS; do
    if [ "$L" = default ]; then unset GPMPC_LIB; else export GPMPC_LIB=$L; fi
    probe=$(timeout -k 10 120 python3 scripts/gemm_loop_probe.py 2>/dev/null | grep '^{')
    out=$(timeout -k 10 300 python3 bench.py --no-cpu --steps 20 2>/dev/null | grep '^{')
    python3 -c "
import json,sys
d=json.loads(sys.argv[2]); k=d['kernels']; c=d['cholesky']; p=json.loads(sys.argv[3])
print(sys.argv[1], d['value'], d['ms_per_step'], {x: (v['ms'], round(v['frac'], 4)) for x, v in k.items()},
      'potrf', {b: v['frac_fp64_peak'] for b, v in c['by_batch'].items()}, 'syrk_potrf', c['syrk_potrf']['frac_fp64_peak'],
      'syrk_fitc', c['syrk_fitc']['frac_fp64_peak'], 'loop', p['frac_min'], p['maxerr'])" "$L" "$out" "$probe" | tee -a "$OUT/ab.log"
  done
done
