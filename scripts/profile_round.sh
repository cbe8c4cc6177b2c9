#!/bin/bash
# Round profiles on the GPU box (run through gpurun from the repo root):
#   trace    rocprofv3 --kernel-trace --stats of the bench's main workload (--no-chol)
#   fulltrace  the same over the full bench (every leg)
#   fetch    --pmc FETCH_SIZE of the bench's main workload (--no-chol: the
#   write    --pmc WRITE_SIZE   1024-landing step only, so per-kernel means are its launches)
#   r6trace  --kernel-trace --stats of the 6-DoF rollouts leg alone at 64 rollouts
#   r6fetch / r6write  its two --pmc passes
# then scripts/pmc_traffic.py -> per-launch HBM bytes per kernel (FETCH x2 per the guide).
# Separate passes: FETCH_SIZE and WRITE_SIZE take separate TCC slots on gfx950.
# Usage: bash scripts/profile_round.sh TAG ["trace fulltrace fetch write r6trace r6fetch r6write"]
set -euo pipefail
TAG=${1:-r1}
PASSES=${2:-trace fulltrace fetch write r6trace r6fetch r6write}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for p in $PASSES; do
  case $p in
    trace) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
             python3 "$ROOT/bench.py" --no-cpu --no-chol > "$OUT/bench_trace.log" 2>&1 ;;
    fulltrace) timeout -k 10 560 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/fulltrace" -o run -- \
             python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu > "$OUT/bench_fulltrace.log" 2>&1 ;;
    fetch) timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
             python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-chol > "$OUT/bench_fetch.log" 2>&1 ;;
    write) timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
             python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-chol > "$OUT/bench_write.log" 2>&1 ;;
    r6trace) BATCHES=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r6trace" -o run -- \
             python3 "$ROOT/scripts/rollouts6_probe.py" > "$OUT/r6_trace.log" 2>&1 ;;
    r6fetch) BATCHES=64 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/r6fetch" -o run -- \
             python3 "$ROOT/scripts/rollouts6_probe.py" > "$OUT/r6_fetch.log" 2>&1 ;;
    r6write) BATCHES=64 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/r6write" -o run -- \
             python3 "$ROOT/scripts/rollouts6_probe.py" > "$OUT/r6_write.log" 2>&1 ;;
  esac
done
cd "$ROOT"
csv() { find "$OUT/$1" -name '*counter_collection.csv' | head -1; }
if [ -d "$OUT/fetch" ] && [ -d "$OUT/write" ]; then
  python3 scripts/pmc_traffic.py "$(csv fetch)" "$(csv write)" "$OUT/pmc_traffic.json"
fi
if [ -d "$OUT/r6fetch" ] && [ -d "$OUT/r6write" ]; then
  python3 scripts/pmc_traffic.py "$(csv r6fetch)" "$(csv r6write)" "$OUT/rollouts6_pmc_traffic.json"
fi
echo "profiles in $OUT"
