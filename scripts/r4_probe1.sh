#!/bin/bash
# Round-4 first measurement pass (through gpurun, from the repo root):
#  1. MFMA-busy / VALU / LDS counters per kernel of the batched potrf at batch 1024 and 256
#     (scripts/pmc_mfma.sh over scripts/potrf_probe.py)
#  2. posterior-GEMM HBM traffic with K* past the 256 MiB Infinity Cache: the bench's main
#     workload at 2048 landings (K* = 2048 x 20 x 1000 x 8 B = 328 MB), FETCH_SIZE and
#     WRITE_SIZE passes -> gpurun_out/prof_b2048/pmc_traffic.json
set -euo pipefail
ROOT=$(pwd)
PROBE_SHAPES=1000x1024 bash scripts/pmc_mfma.sh potrf1024 python3 scripts/potrf_probe.py
PROBE_SHAPES=1000x256 bash scripts/pmc_mfma.sh potrf256 python3 scripts/potrf_probe.py
OUT=$ROOT/gpurun_out/prof_b2048
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$ROOT/bench.py" --landings 2048 --steps 10 --warmup 3 --no-cpu --no-chol \
  > "$OUT/bench.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" --landings 2048 --steps 3 --warmup 1 --no-cpu --no-chol > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" --landings 2048 --steps 3 --warmup 1 --no-cpu --no-chol > "$OUT/write.log" 2>&1
cd "$ROOT"
csv() { find "$OUT/$1" -name '*counter_collection.csv' | head -1; }
python3 scripts/pmc_traffic.py "$(csv fetch)" "$(csv write)" "$OUT/pmc_traffic.json"
echo done
