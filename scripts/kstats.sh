#!/bin/bash
# rocprofv3 kernel-trace stats of a command, top kernels printed:
#   bash scripts/kstats.sh TAG cmd args...   (env passes through)
set -euo pipefail
TAG=$1; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/kstats_$TAG
mkdir -p "$OUT"
ARGS=()
for a in "$@"; do if [ -e "$a" ]; then ARGS+=("$(realpath "$a")"); else ARGS+=("$a"); fi; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- "${ARGS[@]}" > "$OUT/cmd.log" 2>&1
cd "$ROOT"
python3 - "$OUT/run_kernel_stats.csv" <<'PY' | tee "$OUT/top.txt"
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:9.1f} us {float(r["Percentage"]):6.2f}%')
PY
