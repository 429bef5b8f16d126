#!/bin/bash
# r03g: the op-body tests (plain and under ThreadSanitizer) and the resnet50 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03g"
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest -x -v -m gpu --timeout 150 --timeout-method thread tests/test_gpu_op_body.py > "$OUT/pytest_op_body.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/steps.txt"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 240 python -u bench.py --workload resnet50 --no-compare > "$OUT/bench_resnet50.log" 2>&1
