#!/bin/bash
# potrf kernel breakdown under rocprofv3 for the default and a variant env:
#   bash scripts/potrf_ab.sh TAG "ENV=VAL ..." SHAPES
set -euo pipefail
TAG=$1; ENVS=$2; SHAPES=${3:-1000x256}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/potrf_ab_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
env PROBE_SHAPES=$SHAPES $ENVS timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$ROOT/scripts/potrf_probe.py" > "$OUT/probe.log" 2>&1
env PROBE_SHAPES=$SHAPES $ENVS timeout -k 10 200 python3 "$ROOT/scripts/potrf_probe.py" > "$OUT/probe_noprof.log" 2>&1
