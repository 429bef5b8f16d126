#!/bin/bash
# r03i: hunt the op-body hang with the watchdog's state reports, then the TSan op-body probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03i"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
RUNS=6 TAG=r03i/hunt bash tools/gpu_op_body_hunt.sh
TAG=r03i/tsan bash tools/gpu_tsan_probe.sh
echo "tsan rc=$?" >> "$OUT/steps.txt"
