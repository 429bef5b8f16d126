#!/bin/bash
# r03f: bench lines on the current tree (default, fused1000, resnet50), then the round-3 PMC passes
# and the kernel-trace summary of the default command (tools/gpu_pmc_r03.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03f"
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
timeout -k 10 300 python -u bench.py > "$OUT/bench.log" 2>&1 || exit $?
for w in fused1000 resnet50; do
  timeout -k 10 240 python -u bench.py --workload $w --no-compare > "$OUT/bench_$w.log" 2>&1 || exit $?
done
TAG=r03f/pmc bash tools/gpu_pmc_r03.sh
