#!/bin/bash
# early LDS store in the 128-tile loop (MMA_EARLY_LS): parity with it, then A/B against
# ab/libgpmpc_ls0.so (built with -DMMA_EARLY_LS=0): dense loop, potrf, the bench step
set -euo pipefail
mkdir -p gpurun_out/probe8
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "potrf or fit or fitc or exact or trsm or simple3dof or surfaces or fleet_closed or posterior or syrk" \
  > gpurun_out/probe8/tests.log 2>&1
tail -1 gpurun_out/probe8/tests.log
for v in new ls0 bar1; do
  L=""; [ $v != new ] && L=ab/libgpmpc_$v.so
  GPMPC_LIB=$L timeout -k 10 120 python3 -u scripts/gemm_loop_probe.py > gpurun_out/probe8/loop_$v.log 2>&1
  GPMPC_LIB=$L PROBE_SHAPES=1000x256,1000x1024,1000x64 timeout -k 10 300 python3 -u scripts/potrf_probe.py \
    > gpurun_out/probe8/potrf_$v.log 2>&1
  GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 3 --no-cpu --no-chol \
    > gpurun_out/probe8/bench_$v.log 2>&1
  echo "== $v"; cat gpurun_out/probe8/loop_$v.log; grep -v amdgpu gpurun_out/probe8/potrf_$v.log
  grep '"metric"' gpurun_out/probe8/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
