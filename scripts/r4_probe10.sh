#!/bin/bash
# solve-only first block column with 16-byte loads (k_gemm128_updsolve<false, true>) and the
# last block column's diagonal update on k_syrk128_diag: parity, timing, per-launch trace
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe10
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "potrf or lml or fit or exact" > gpurun_out/probe10/tests.log 2>&1
tail -1 gpurun_out/probe10/tests.log
PROBE_SHAPES=1000x256,1000x512,1000x1024,2000x256 timeout -k 10 300 python3 -u scripts/potrf_probe.py \
  > gpurun_out/probe10/potrf.log 2>&1
grep -v amdgpu gpurun_out/probe10/potrf.log
PROBE_SHAPES=1000x1024 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/probe10/kt -o kt \
  --output-format csv -- python3 -u scripts/potrf_probe.py > gpurun_out/probe10/kt.log 2>&1
echo done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rollouts6.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "config5" > gpurun_out/probe10/r6tests.log 2>&1
tail -3 gpurun_out/probe10/r6tests.log
cd /tmp && timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/probe10/counters.txt 2>&1 || true
cd $GRAFT_REPO_ROOT
grep -o "SQ_[A-Z_]*LDS[A-Z_]*" gpurun_out/probe10/counters.txt | sort -u > gpurun_out/probe10/lds_counters.txt || true
for v in new prio; do
  L=""; [ $v != new ] && L=ab/libgpmpc_$v.so
  GPMPC_LIB=$L timeout -k 10 120 python3 -u scripts/gemm_loop_probe.py > gpurun_out/probe10/loop_$v.log 2>&1
  GPMPC_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 3 --no-cpu --no-chol \
    > gpurun_out/probe10/bench_$v.log 2>&1
  echo "== $v"; cat gpurun_out/probe10/loop_$v.log
  grep '"metric"' gpurun_out/probe10/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
echo "== batch 64-192: right-looking (default) vs left-looking fused (OB 1024, fuse from 1 workgroup)"
PROBE_SHAPES=1000x64,1000x128,1000x192 timeout -k 10 200 python3 -u scripts/potrf_probe.py 2>&1 | grep -v amdgpu
GPMPC_POTRF_OB=1024 GPMPC_POTRF_FUSE_MIN=1 PROBE_SHAPES=1000x64,1000x128,1000x192 timeout -k 10 200 \
  python3 -u scripts/potrf_probe.py 2>&1 | grep -v amdgpu
