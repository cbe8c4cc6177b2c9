#!/bin/bash
# Gram rows by scalar loads (GRAM_SCALAR_ROWS) against the LDS-staged rows (ab/libgpmpc_g0.so)
set -euo pipefail
mkdir -p gpurun_out/probe19
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "gram or posterior or exact or fleet_closed or surfaces or simple3dof" > gpurun_out/probe19/tests.log 2>&1
tail -1 gpurun_out/probe19/tests.log
for v in new g0 new g0; do
  L=""; [ $v != new ] && L=ab/libgpmpc_$v.so
  GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 3 --no-cpu --no-chol > gpurun_out/probe19/bench_$v.log 2>&1
  echo "== $v $(grep '"metric"' gpurun_out/probe19/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['qp_status']['admm_iterations'])")"
done
