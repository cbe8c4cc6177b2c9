#!/bin/bash
# batch-64 potrf (right-looking): per-kernel time
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe16
PROBE_SHAPES=1000x64 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/probe16/kt -o kt \
  --output-format csv -- python3 -u scripts/potrf_probe.py > gpurun_out/probe16/kt.log 2>&1
python3 - <<'P'
import csv
for r in csv.DictReader(open('gpurun_out/probe16/kt/kt_kernel_stats.csv')):
    n = r['Name']
    if any(k in n for k in ('potrf', 'gemm', 'syrk', 'psolve')) and not n.startswith('Cijk'):
        print(n[:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), round(float(r['TotalDurationNs']) / 4e6, 3))
P
