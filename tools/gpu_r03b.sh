#!/bin/bash
# r03b: allreduce_grads' C++ list helper (tests + bench gradient_api legs), the pack kernel's
# launch-size ceiling, and the fused host path's phase split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03b"
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
step() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> "$OUT/steps.txt"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> "$OUT/steps.txt"; return $rc; }
step pytest_grads 400 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_allreduce.py tests/test_gpu_rccl_procs.py -k "grads or fusion or fused or flat" || exit 1
step bench_fused1000 240 python -u bench.py --workload fused1000 --no-compare || exit 1
step bench_resnet50 240 python -u bench.py --workload resnet50 --no-compare || exit 1
step pack_ceiling 240 python -u tools/pack_ceiling.py 7 || exit 1
TIPS_FUSION_THRESHOLD=2147483648 step pack_ceiling_sizes 240 python -u tools/pack_ceiling.py 7 || exit 1
TIPS_HOST_TRACE=1 step host_probe 200 python -u tools/host_probe.py || exit 1
exit 0
