#!/bin/bash
# r03z: list enqueues remember the device allocations they met (PtrRanges) and dev_list's cap -
# the named / negotiation / op-body / gradient-list GPU tests, a short op-body hunt, and the
# negotiated1000 bench line twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03z"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
timeout -k 10 700 python -u -m pytest -x -q -m gpu --timeout 250 --timeout-method thread tests/test_gpu_op_body.py tests/test_gpu_rccl_procs.py tests/test_gpu_allreduce.py -k "op_body or named or negotiat or control_plane or broadcast or allgather or routed or sync or enqueue_n or grads or fused_list or flat" > "$OUT/pytest_neg.log" 2>&1 || exit $?
RUNS=4 TAG=r03z/hunt bash tools/gpu_op_body_hunt.sh
for k in 1 2; do timeout -k 10 200 python -u bench.py --workload negotiated1000 --no-compare > "$OUT/bench_negotiated1000_$k.log" 2>&1 || exit $?; done
