#!/bin/bash
# balanced diagonal-block SYRK in the left-looking potrf (GPMPC_SYRK_DIAG): parity, then
# batch 256 / 512 / 1024 with it on / off, and a kernel trace of batch 1024
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe9
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "potrf or lml or fit or exact" > gpurun_out/probe9/tests.log 2>&1
tail -1 gpurun_out/probe9/tests.log
for v in 1 0; do
  GPMPC_SYRK_DIAG=$v PROBE_SHAPES=1000x256,1000x512,1000x1024 timeout -k 10 300 python3 -u scripts/potrf_probe.py \
    > gpurun_out/probe9/potrf_sd$v.log 2>&1
  echo "== $v"; grep -v amdgpu gpurun_out/probe9/potrf_sd$v.log
done
PROBE_SHAPES=1000x1024 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/probe9/kt -o kt \
  --output-format csv -- python3 -u scripts/potrf_probe.py > gpurun_out/probe9/kt.log 2>&1
grep -E "syrk128|updsolve|diag128|k_gemm128" gpurun_out/probe9/kt/kt_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
