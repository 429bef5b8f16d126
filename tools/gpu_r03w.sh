#!/bin/bash
# r03w: bench.py's N = 4 line on config 5 (214 gradients, fused) over 4 RCCL ranks sharing the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03w"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
TIPS_BENCH_FAKE_HOSTS=1 timeout -k 10 700 python -u bench.py --gpus 4 --workload resnet50 --steps 5 --warmup 2 > "$OUT/rehearsal_n4_resnet50.log" 2>&1
