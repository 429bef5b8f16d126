#!/bin/bash
# r03h: the TSan op-body probe, then the whole GPU suite and smoke on the current tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03h"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
TAG=r03h/tsan bash tools/gpu_tsan_probe.sh
echo "tsan probe rc=$?" >> "$OUT/steps.txt"
timeout -k 10 800 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread --deselect tests/test_gpu_op_body.py::test_op_body_under_tsan > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/steps.txt"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
