#!/bin/bash
# Round profiles on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of the full bench (every leg: the
#      summary committed under profiles/)
#   2. two separate --pmc passes (FETCH_SIZE, WRITE_SIZE: separate TCC slots on gfx950)
#   3. scripts/pmc_traffic.py -> per-launch HBM bytes per kernel (FETCH x2 per the guide)
# Usage: bash scripts/profile_round.sh TAG ["trace fetch write"]
set -euo pipefail
TAG=${1:-r1}
PASSES=${2:-trace fetch write}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for p in $PASSES; do
  case $p in
    trace) timeout -k 10 560 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
             python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu > "$OUT/bench_trace.log" 2>&1 ;;
    fetch) timeout -k 10 560 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
             python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$OUT/bench_fetch.log" 2>&1 ;;
    write) timeout -k 10 560 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
             python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$OUT/bench_write.log" 2>&1 ;;
  esac
done
cd "$ROOT"
if [ -d "$OUT/fetch" ] && [ -d "$OUT/write" ]; then
  python3 scripts/pmc_traffic.py "$(find "$OUT/fetch" -name '*counter_collection.csv' | head -1)" \
    "$(find "$OUT/write" -name '*counter_collection.csv' | head -1)" "$OUT/pmc_traffic.json"
fi
echo "profiles in $OUT"
