#!/bin/bash
# r03t: more evidence on the final tree - the op-body hunt (20 runs, default build), then the whole
# GPU suite once more.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03t"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
RUNS=20 TAG=r03t/hunt bash tools/gpu_op_body_hunt.sh
timeout -k 10 800 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
echo "pytest rc=$?" >> "$OUT/steps.txt"
