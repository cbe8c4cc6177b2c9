#!/bin/bash
# config-5 rollouts parity, s_setprio A/B on the 128-tile loop, small-batch left-looking potrf,
# the LDS counter names this rocprofv3 offers
set -euo pipefail
mkdir -p gpurun_out/probe11
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rollouts6.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "config5" > gpurun_out/probe11/r6tests.log 2>&1
tail -1 gpurun_out/probe11/r6tests.log
for v in new prio; do
  L=""; [ $v != new ] && L=ab/libgpmpc_$v.so
  GPMPC_LIB=$L timeout -k 10 120 python3 -u scripts/gemm_loop_probe.py > gpurun_out/probe11/loop_$v.log 2>&1
  GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 3 --no-cpu --no-chol \
    > gpurun_out/probe11/bench_$v.log 2>&1
  echo "== $v"; cat gpurun_out/probe11/loop_$v.log
  grep '"metric"' gpurun_out/probe11/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
echo "== batch 64-192: right-looking (default) vs left-looking fused (OB 1024, fuse from 1 workgroup)"
PROBE_SHAPES=1000x64,1000x128,1000x192 timeout -k 10 200 python3 -u scripts/potrf_probe.py > gpurun_out/probe11/small_rl.log 2>&1
GPMPC_POTRF_OB=1024 GPMPC_POTRF_FUSE_MIN=1 PROBE_SHAPES=1000x64,1000x128,1000x192 timeout -k 10 200 \
  python3 -u scripts/potrf_probe.py > gpurun_out/probe11/small_ll.log 2>&1
grep -h "batch" gpurun_out/probe11/small_rl.log gpurun_out/probe11/small_ll.log
cd /tmp && timeout -k 10 60 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/probe11/counters.txt" 2>&1 || true
echo done
