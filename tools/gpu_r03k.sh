#!/bin/bash
# r03k: which ingredient the op-body hang needs - the hunt (up to 12 runs, stop at the first hang)
# with replayed plans off, with 16 hardware queues per process, and with non-blocking streams and no
# legacy-null-stream copies in the test program.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03k"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
TIPS_GRAPHS=0 RUNS=12 TAG=r03k/nographs bash tools/gpu_op_body_hunt.sh
OP_BODY_NONBLOCKING=1 RUNS=12 TAG=r03k/nonblocking bash tools/gpu_op_body_hunt.sh
GPU_MAX_HW_QUEUES=16 RUNS=12 TAG=r03k/hwq16 bash tools/gpu_op_body_hunt.sh
