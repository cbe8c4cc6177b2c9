#!/bin/bash
# stream-K SYRK with the diagonal tiles on k_syrk128_diag: parity, then the config-5 FITC SYRK
set -euo pipefail
mkdir -p gpurun_out/probe17
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "syrk or fitc or structured or vfe or potrf" > gpurun_out/probe17/tests.log 2>&1
tail -1 gpurun_out/probe17/tests.log
for v in 1 0 1 0; do
  echo "sk_syrk_diag=$v $(GPMPC_SK_SYRK_DIAG=$v timeout -k 10 120 python3 -u scripts/syrk_probe.py 2>/dev/null)"
done
