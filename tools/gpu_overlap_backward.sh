#!/bin/bash
# DistributedOptimizer's allreduce during vs after backward, 2 real RCCL ranks on the box's GPU,
# from rocprofv3 kernel traces (tools/overlap_backward.py). Every rank is its own
# rocprofv3 process started from this shell (no process under the profiler starts another), each
# under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-ovlbwd}"
mkdir -p "$OUT"
export TMPDIR=/tmp
port=29611
for ov in 0 1; do
  d="$OUT/ov$ov"
  pids=()
  for r in 0 1; do
    TIPS_OVERLAP_BACKWARD=$ov timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$d/rank$r" \
      -- python3 tools/overlap_backward.py worker $r 2 $port 5 > "$OUT/ov${ov}_rank$r.log" 2>&1 &
    pids+=($!)
  done
  for p in "${pids[@]}"; do
    wait "$p" || exit $?
  done
  python3 tools/overlap_backward.py report "$d" "TIPS_OVERLAP_BACKWARD=$ov" >> "$OUT/overlap_backward.jsonl" || exit $?
  cat "$OUT"/ov${ov}_rank*.log | grep '^{' >> "$OUT/runs.jsonl"
  port=$((port + 1))
done
exit 0
