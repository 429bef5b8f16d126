#!/bin/bash
# r03x: the enqueue wake change - negotiation GPU tests (named requests over RCCL ranks, op-body),
# a short op-body hunt, and the negotiated1000 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03x"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 250 --timeout-method thread tests/test_gpu_op_body.py tests/test_gpu_rccl_procs.py tests/test_gpu_allreduce.py -k "op_body or named or negotiat or control_plane or broadcast or allgather or routed or sync" > "$OUT/pytest_neg.log" 2>&1 || exit $?
RUNS=8 TAG=r03x/hunt bash tools/gpu_op_body_hunt.sh
for k in 1 2; do timeout -k 10 200 python -u bench.py --workload negotiated1000 --no-compare > "$OUT/bench_negotiated1000_$k.log" 2>&1 || exit $?; done
