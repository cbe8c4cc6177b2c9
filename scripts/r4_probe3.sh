#!/bin/bash
# MFMA busy per kernel of the bench's main workload; the column-grouped posterior mapping
# (GPMPC_POST_XCD=1) at 2048 landings: time and HBM traffic; the configs[1] fit
set -euo pipefail
ROOT=$(pwd)
bash scripts/pmc_mfma.sh main1024 python3 bench.py --steps 5 --warmup 2 --no-cpu --no-chol
OUT=$ROOT/gpurun_out/prof_b2048_postxcd
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
GPMPC_POST_XCD=1 timeout -k 10 300 python3 "$ROOT/bench.py" --landings 2048 --steps 10 --warmup 3 --no-cpu --no-chol \
  > "$OUT/bench.log" 2>&1
GPMPC_POST_XCD=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" --landings 2048 --steps 3 --warmup 1 --no-cpu --no-chol > "$OUT/fetch.log" 2>&1
GPMPC_POST_XCD=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" --landings 2048 --steps 3 --warmup 1 --no-cpu --no-chol > "$OUT/write.log" 2>&1
cd "$ROOT"
csv() { find "$OUT/$1" -name '*counter_collection.csv' | head -1; }
python3 scripts/pmc_traffic.py "$(csv fetch)" "$(csv write)" "$OUT/pmc_traffic.json"
timeout -k 10 300 python3 -c "
import json, bench
from gp_mpc_rocket_landing_amd import _lib
print(json.dumps(bench.simple3dof_gp_bench(_lib.Context(0), cpu=False)))" > gpurun_out/fit_bench.log 2>&1
echo done
