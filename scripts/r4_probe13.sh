#!/bin/bash
# the fleet's control kernel at 256 threads per landing (one item per thread, four waves,
# ab/libgpmpc_t256.so built with -DFQ_T=256) against the 128-thread default: parity, bench
set -euo pipefail
mkdir -p gpurun_out/probe13
GPMPC_LIB=ab/libgpmpc_t256.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fleet_parity.py -m gpu -x -v -s \
  --timeout 300 --timeout-method thread -k "not mc1024_every_step" > gpurun_out/probe13/tests.log 2>&1 || true
tail -3 gpurun_out/probe13/tests.log
for v in new t256; do
  L=""; [ $v != new ] && L=ab/libgpmpc_$v.so
  GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 3 --no-cpu --no-chol \
    > gpurun_out/probe13/bench_$v.log 2>&1
  echo "== $v"
  grep '"metric"' gpurun_out/probe13/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['outcomes'], d['qp_status']['admm_iterations'])"
done
