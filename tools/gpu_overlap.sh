#!/bin/bash
# Transfer/sum overlap of the ring and direct schedules at config 3's shape (8 virtual ranks x 1 GiB),
# from rocprofv3 kernel traces (run on the GPU box via gpurun).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-overlap}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for sched in ring direct; do
  for tr in 1 0; do
    d="$OUT/${sched}_t$tr"
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$d" -o trace \
      -- python3 tools/overlap_profile.py $sched $tr 3 > "$OUT/${sched}_t$tr.log" 2>&1 || exit $?
    f=$(find "$d" -name '*kernel_trace.csv' | head -1)
    python3 tools/overlap_report.py "$f" "${sched} transport=$tr" >> "$OUT/overlap.jsonl" || exit $?
    grep '^{' "$OUT/${sched}_t$tr.log" >> "$OUT/runs.jsonl"
  done
done
exit 0
