#!/bin/bash
# A/B measurements over library builds and environment switches (GPU box, repo root).
#   bash scripts/ab.sh build NAME SRC.hip "-DFLAG=1 ..."
#        one translation unit rebuilt with extra flags, linked against the other objects of
#        the current build -> ab/libgpmpc_NAME.so (loaded through GPMPC_LIB)
#   bash scripts/ab.sh run OUTDIR WORKLOAD "SETTINGS" [reps]
#        WORKLOAD: main (the bench's main workload, --no-chol), full (+ the Cholesky legs and
#        the 128-tile loop probe), chol (the Cholesky leg), syrk_fitc, rollouts6 (64 / 512)
#        SETTINGS: "-" (as built), VAR=value (environment), NAME or path.so (ab/libgpmpc_NAME.so)
#        One line per run, appended to OUTDIR/ab.log.
set -euo pipefail
MODE=$1; shift
if [ "$MODE" = build ]; then
  NAME=$1; SRC=$2; XF=${3:-}
  C=gp_mpc_rocket_landing_amd/csrc
  mkdir -p ab
  make -s -C $C >/dev/null
  OBJ=$(basename "$SRC" .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC $XF -c $C/$SRC -o /tmp/ab_${NAME}_$OBJ.o
  OTHERS=$(ls $C/build/*.o | grep -v "/$OBJ.o$")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OTHERS /tmp/ab_${NAME}_$OBJ.o -ldl -o ab/libgpmpc_$NAME.so
  echo "ab/libgpmpc_$NAME.so"
  exit 0
fi
OUT=$1; WL=$2; SETS=$3; REPS=${4:-1}
mkdir -p "$OUT"
run() {
  case $WL in
    main) timeout -k 10 300 python3 bench.py --no-cpu --no-chol --steps 20 --warmup 5 ;;
    full) echo "LOOP $(timeout -k 10 120 python3 scripts/probe.py gemm_loop | grep '^{')"
          timeout -k 10 300 python3 bench.py --no-cpu --steps 20 ;;
    chol) timeout -k 10 200 python3 scripts/probe.py chol ;;
    syrk_fitc) timeout -k 10 120 python3 scripts/probe.py syrk_fitc ;;
    rollouts6) timeout -k 10 300 python3 scripts/probe.py rollouts6 64,512 ;;
    *) echo "unknown workload $WL" >&2; exit 2 ;;
  esac
}
SUMMARY=$(cat <<'PY'
import json, sys
wl, lab = sys.argv[1], sys.argv[2]
lines = sys.stdin.read().splitlines()
d = json.loads([l for l in lines if l.startswith("{")][-1])
if wl in ("main", "full"):
    s = [d["value"], d["ms_per_step"], {x: (v["ms"], round(v["frac"], 4)) for x, v in d["kernels"].items()}]
    if wl == "full":
        c = d["cholesky"]
        loop = json.loads([l for l in lines if l.startswith("LOOP ")][0][5:])
        s += ["potrf", {b: v["frac_fp64_peak"] for b, v in c["by_batch"].items()},
              "syrk_potrf", c["syrk_potrf"]["frac_fp64_peak"], "syrk_fitc", c["syrk_fitc"]["frac_fp64_peak"],
              "loop", loop["frac_min"], loop["maxerr"]]
elif wl == "chol":
    s = [{b: v["frac_fp64_peak"] for b, v in d["by_batch"].items()}, "syrk_potrf",
         d["syrk_potrf"]["frac_fp64_peak"], "syrk_fitc", d["syrk_fitc"]["frac_fp64_peak"]]
elif wl == "rollouts6":
    s = [d["64"]["ms_per_step"], d["512"]["ms_per_step"], d["64"]["launched_steps"], d["512"]["launched_steps"]]
else:
    s = [d]
print(lab, *s)
PY
)
summary() { python3 -c "$SUMMARY" "$WL" "$1"; }
for r in $(seq 1 "$REPS"); do
  for S in $SETS; do
    if [ "$S" = - ]; then out=$(run 2>/dev/null)
    elif [[ "$S" == *=* ]]; then out=$(export "$S"; run 2>/dev/null)
    elif [[ "$S" == *.so ]]; then out=$(export GPMPC_LIB=$S; run 2>/dev/null)
    else out=$(export GPMPC_LIB=ab/libgpmpc_$S.so; run 2>/dev/null); fi
    echo "$out" | summary "$S" | tee -a "$OUT/ab.log"
  done
done
