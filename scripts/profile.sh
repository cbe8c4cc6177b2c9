#!/bin/bash
# Profiles and checks on the GPU box (through gpurun, from the repo root).  Output under
# gpurun_out/TAG/; copy what is to be kept into profiles/.
#   bash scripts/profile.sh TAG "PASSES" [-- command ...]
# Passes (each under its own time limit; --pmc passes alone, counters per the guide's limits):
#   tests      the GPU suite (PYTEST_ARGS: extra pytest arguments, e.g. -k EXPR or test files)
#   surface    the two drop-in surface legs (probe.py surface / surface6) -> surface.json, surface6.json
#   bench      the default bench line -> bench.json
#   trace      --kernel-trace --stats of the bench's main workload (--no-chol)
#   fulltrace  the same over the full bench (every leg)
#   fetch / write   --pmc FETCH_SIZE / WRITE_SIZE of the main workload -> pmc_traffic.json
#   r6trace / r6fetch / r6write   the same for the configs[4] rollouts leg at 64 rollouts
#   r6mem      two --pmc passes of memory-pipeline counters over the rollouts leg (k_r6_* sums)
#   mfma       --pmc MFMA busy / clock / waits of the command (default: the main workload)
#   kstats     --kernel-trace --stats of the command, top kernels
#   pmc        one --pmc pass of the counters in $PMC over the command (default: the main
#              workload), per-kernel means of the kernels starting with $PMC_PREFIX (default k_)
set -euo pipefail
TAG=$1; PASSES=$2; shift 2
[ "${1:-}" = "--" ] && shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
CMD=()
for a in "$@"; do if [ -e "$a" ]; then CMD+=("$(realpath "$a")"); else CMD+=("$a"); fi; done
MAIN=(python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-chol)
R6=(python3 "$ROOT/scripts/probe.py" rollouts6 64)
csv() { find "$OUT/$1" -name "*$2.csv" | head -1; }
prof() {  # prof LIMIT DIR rocprofv3-options... -- program...
  local lim=$1 dir=$2; shift 2
  (cd /tmp && TMPDIR=/tmp timeout -k 10 "$lim" rocprofv3 "$@" > "$OUT/$dir.log" 2>&1)
}
for p in $PASSES; do
  case $p in
    tests) timeout -k 10 "${GT_TIMEOUT:-900}" python3 -u -m pytest -m gpu -x -v --timeout 300 \
             --timeout-method thread ${PYTEST_ARGS:-tests} > "$OUT/tests.log" 2>&1
           tail -3 "$OUT/tests.log" ;;
    surface) timeout -k 10 300 python3 scripts/probe.py surface > "$OUT/surface.json" 2>"$OUT/surface.err"
           timeout -k 10 300 python3 scripts/probe.py surface6 > "$OUT/surface6.json" 2>"$OUT/surface6.err"
           cat "$OUT/surface.json" "$OUT/surface6.json" ;;
    bench) timeout -k 10 360 python3 bench.py > "$OUT/bench.log" 2>&1
           grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json" ;;
    trace) prof 300 trace --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
             python3 "$ROOT/bench.py" --no-cpu --no-chol ;;
    fulltrace) prof 560 fulltrace --kernel-trace --stats --output-format csv -d "$OUT/fulltrace" -o run -- \
             python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu ;;
    fetch) prof 300 fetch --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- "${MAIN[@]}" ;;
    write) prof 300 write --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- "${MAIN[@]}" ;;
    r6trace) prof 300 r6trace --kernel-trace --stats --output-format csv -d "$OUT/r6trace" -o run -- "${R6[@]}" ;;
    r6fetch) prof 300 r6fetch --pmc FETCH_SIZE --output-format csv -d "$OUT/r6fetch" -o run -- "${R6[@]}" ;;
    r6write) prof 300 r6write --pmc WRITE_SIZE --output-format csv -d "$OUT/r6write" -o run -- "${R6[@]}" ;;
    r6mem)
      (cd /tmp && TMPDIR=/tmp timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD \
         SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE \
         --output-format csv -d "$OUT/r6mem1" -o run -- "${R6[@]}" > "$OUT/r6mem1.log" 2>&1)
      (cd /tmp && TMPDIR=/tmp timeout -s KILL 240 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum \
         TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum \
         GRBM_GUI_ACTIVE --output-format csv -d "$OUT/r6mem2" -o run -- "${R6[@]}" > "$OUT/r6mem2.log" 2>&1)
      for q in r6mem1 r6mem2; do python3 scripts/pmc.py sum "$(csv $q counter_collection)" k_r6_ > "$OUT/$q.txt"; done ;;
    mfma)
      [ ${#CMD[@]} -gt 0 ] || CMD=("${MAIN[@]}")
      (cd /tmp && TMPDIR=/tmp timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
         SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_F64 \
         SQ_INSTS_LDS --kernel-trace --output-format csv -d "$OUT/mfma" -o run -- "${CMD[@]}" > "$OUT/mfma.log" 2>&1)
      python3 scripts/pmc.py mfma "$(csv mfma counter_collection)" "$(csv mfma kernel_trace)" > "$OUT/mfma.txt" ;;
    kstats)
      prof 400 kstats --kernel-trace --stats --output-format csv -d "$OUT/kstats" -o run -- "${CMD[@]}"
      python3 scripts/pmc.py top "$(csv kstats kernel_stats)" | tee "$OUT/kstats.txt" ;;
    pmc)
      [ ${#CMD[@]} -gt 0 ] || CMD=("${MAIN[@]}")
      (cd /tmp && TMPDIR=/tmp timeout -s KILL 300 rocprofv3 --pmc $PMC --output-format csv -d "$OUT/pmc" -o run \
         -- "${CMD[@]}" > "$OUT/pmc.log" 2>&1)
      python3 scripts/pmc.py sum "$(csv pmc counter_collection)" "${PMC_PREFIX:-k_}" > "$OUT/pmc.txt" ;;
    *) echo "unknown pass $p" >&2; exit 2 ;;
  esac
done
if [ -d "$OUT/fetch" ] && [ -d "$OUT/write" ]; then
  python3 scripts/pmc.py traffic "$(csv fetch counter_collection)" "$(csv write counter_collection)" "$OUT/pmc_traffic.json"
fi
if [ -d "$OUT/r6fetch" ] && [ -d "$OUT/r6write" ]; then
  python3 scripts/pmc.py traffic "$(csv r6fetch counter_collection)" "$(csv r6write counter_collection)" \
    "$OUT/rollouts6_pmc_traffic.json"
fi
echo "output in $OUT"
