#!/bin/bash
# r03d: the fused host path's DMA copy trace, then the N = 2 one-GPU rehearsal of bench.py's
# default N > 1 line (2 RCCL ranks, socket transport).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03d"
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
PIECES="8388608 33554432" TAG=r03d bash tools/gpu_host_copy_trace.sh || exit $?
TIPS_BENCH_FAKE_HOSTS=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 5 --warmup 2 > "$OUT/rehearsal_n2.log" 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u tools/pack_ceiling.py 7 > "$OUT/pack_ceiling.jsonl" 2> "$OUT/pack_ceiling.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_pack" -o run \
    -- python3 tools/pack_ceiling.py 3 > "$OUT/prof_pack.log" 2>&1
