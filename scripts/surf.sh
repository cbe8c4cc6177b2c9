# The GPU suite (or PYTEST_ARGS) and the drop-in surface timing, on the GPU box.
set -e
timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-tests} > gpurun_out/surf_tests.log 2>&1
tail -3 gpurun_out/surf_tests.log
timeout -k 10 300 python3 scripts/surf_run.py 2 > gpurun_out/surf.log 2>&1
tail -1 gpurun_out/surf.log
