#!/bin/bash
# r03e: the fused host path with a second H2D stream (host_probe --streams), and the DMA copy
# trace at the default 16 MiB pieces with one and two H2D streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03e"
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
TIPS_HOST_TRACE=1 timeout -k 10 300 python -u tools/host_probe.py --streams > "$OUT/host_probe_streams.log" 2>&1 || exit $?
PIECES=16777216 TAG=r03e/one bash tools/gpu_host_copy_trace.sh || exit $?
TIPS_HOST_H2D_STREAMS=2 PIECES=16777216 TAG=r03e/two bash tools/gpu_host_copy_trace.sh || exit $?
TIPS_HOST_H2D_STREAMS=2 timeout -k 10 240 python -u bench.py --workload resnet50 --no-compare > "$OUT/bench_resnet50_two.log" 2>&1
