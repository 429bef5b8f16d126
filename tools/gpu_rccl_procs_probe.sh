#!/bin/bash
# The multi-process RCCL-rank tests alone, verbose, each job capped at TIPS_TEST_JOB_TIMEOUT s (a hung job
# then dumps every rank's Python stacks into the failure); a heartbeat file keeps the call visibly alive.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-rprobe}"
mkdir -p "$OUT"
export TMPDIR=/tmp TIPS_TEST_JOB_TIMEOUT=${TIPS_TEST_JOB_TIMEOUT:-150}
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
HB=$!
timeout -k 10 ${PROBE_TIMEOUT:-900} python -u -m pytest tests/test_gpu_rccl_procs.py -x -v -m gpu --timeout 400 \
  --timeout-method thread -k "${PYTEST_K:-gpu}" > "$OUT/pytest.log" 2>&1
rc=$?
kill $HB
exit $rc
