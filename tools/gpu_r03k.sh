#!/bin/bash
# r03k: which ingredient the op-body hang needs, and whether the fix holds - the hunt (up to 12 runs,
# stop at the first hang) with replayed plans off, with the replay host-order wait (the default
# build), and without it (the control).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03k"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
RUNS=12 TAG=r03k/fix bash tools/gpu_op_body_hunt.sh
TIPS_GRAPHS=0 RUNS=12 TAG=r03k/nographs bash tools/gpu_op_body_hunt.sh
TIPS_REPLAY_HOST_ORDER=0 RUNS=12 TAG=r03k/control bash tools/gpu_op_body_hunt.sh
