#!/bin/bash
# fleet control kernel with the bound-row y / z / delta y as per-slot scalars (no scratch
# array): parity (fleet tests without the long step-locked run), bench, PMC traffic
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe15
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fleet_parity.py tests/test_gpu_surfaces.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "not mc1024_every_step" > gpurun_out/probe15/tests.log 2>&1
tail -1 gpurun_out/probe15/tests.log
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 3 --no-cpu --no-chol > gpurun_out/probe15/bench$r.log 2>&1
  grep '"metric"' gpurun_out/probe15/bench$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['qp_status']['admm_iterations'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/probe15/write" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-chol > "$GRAFT_REPO_ROOT/gpurun_out/probe15/w.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/probe15/fetch" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-chol > "$GRAFT_REPO_ROOT/gpurun_out/probe15/f.log" 2>&1
cd "$GRAFT_REPO_ROOT"
python3 scripts/pmc_traffic.py "$(find gpurun_out/probe15/fetch -name '*counter_collection.csv' | head -1)" \
  "$(find gpurun_out/probe15/write -name '*counter_collection.csv' | head -1)" gpurun_out/probe15/pmc_traffic.json
python3 -c "import json; d=json.load(open('gpurun_out/probe15/pmc_traffic.json'))['kernels']; print({k: round(v['traffic_bytes']/1e6, 2) for k, v in d.items() if 'control' in k or 'gemm128' in k})"
