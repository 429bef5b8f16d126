#!/bin/bash
# bench.py's whole N > 1 path at N = 8 on the box's one GPU (8 RCCL ranks, socket transport:
# TIPS_BENCH_FAKE_HOSTS=1), with a heartbeat file while the long comparisons run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-n8}"
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
HB=$!
TIPS_BENCH_FAKE_HOSTS=1 timeout -k 10 ${N8_TIMEOUT:-1000} python -u bench.py --gpus 8 --steps 3 --warmup 1 \
  ${BENCH_ARGS:-} > "$OUT/rehearsal_n8.log" 2>&1
rc=$?
kill $HB
exit $rc
