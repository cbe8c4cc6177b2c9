#!/bin/bash
# batch-1024 / 256 potrf (fused left-looking path): per-launch kernel trace and the MFMA PMC pass
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe5
for b in 1024 256; do
  PROBE_SHAPES=1000x$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/probe5/kt$b \
    -o kt --output-format csv -- python3 -u scripts/potrf_probe.py > gpurun_out/probe5/kt$b.log 2>&1
  PROBE_SHAPES=1000x$b bash scripts/pmc_mfma.sh potrf${b}_fused python3 scripts/potrf_probe.py \
    > gpurun_out/probe5/pmc$b.txt 2>&1
done
echo done
