#!/bin/bash
# Round-end check on the GPU box, part B: kernel traces and PMC traffic of the main
# workload, the full bench and the 6-DoF leg (scripts/profile_round.sh), then the MFMA
# utilisation pass of the main workload (scripts/pmc_mfma.sh).  Usage: bash scripts/r5_final_b.sh TAG
set -euo pipefail
TAG=${1:-r5final}
bash scripts/profile_round.sh "$TAG" "trace fulltrace fetch write r6trace r6fetch r6write"
bash scripts/pmc_mfma.sh "${TAG}_main1024" python3 bench.py --steps 5 --warmup 2 --no-cpu --no-chol
