#!/bin/bash
# r03m: the op-body tests (plain and under ThreadSanitizer) after the static fix, then the N = 8
# one-GPU rehearsal of bench.py's default N > 1 line (8 RCCL ranks, socket transport).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03m"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest -x -v -m gpu --timeout 250 --timeout-method thread tests/test_gpu_op_body.py > "$OUT/pytest_op_body.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/steps.txt"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
TAG=r03m N8_TIMEOUT=700 bash tools/gpu_rehearsal_n8.sh
echo "n8 rc=$?" >> "$OUT/steps.txt"
