#!/bin/bash
# posterior on 128 x 64 single-buffer tiles (GPMPC_POST_T64=1): parity, then the step A/B
set -euo pipefail
mkdir -p gpurun_out/probe20
GPMPC_POST_T64=1 timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "posterior or exact or fleet_closed or fleet_steps or surfaces or simple3dof or predict" > gpurun_out/probe20/tests.log 2>&1
tail -1 gpurun_out/probe20/tests.log
for v in 1 0 1 0; do
  GPMPC_POST_T64=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 3 --no-cpu --no-chol > gpurun_out/probe20/bench_$v.log 2>&1
  echo "== t64=$v $(grep '"metric"' gpurun_out/probe20/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['qp_status']['admm_iterations'])")"
done
