#!/bin/bash
# r03j: hunt the op-body hang again, now with every thread's stack at 60 s; then the TSan probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03j"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
TAG=r03j/tsan bash tools/gpu_tsan_probe.sh
echo "tsan rc=$?" >> "$OUT/steps.txt"
RUNS=8 TAG=r03j/hunt bash tools/gpu_op_body_hunt.sh
