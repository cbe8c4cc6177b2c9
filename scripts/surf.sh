set -e
timeout -k 10 300 python3 -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_gpu_uprop.py > gpurun_out/uprop_tests.log 2>&1
tail -3 gpurun_out/uprop_tests.log
timeout -k 10 300 python3 -c "
import json, bench
from gp_mpc_rocket_landing_amd import _lib
ctx = _lib.default_context()
print(json.dumps(bench.surface_single_landing_bench(ctx)))
" > gpurun_out/surf.log 2>&1
tail -2 gpurun_out/surf.log
