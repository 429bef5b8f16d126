#!/bin/bash
# The 2-input sum's leading launch shapes / store policies (tools/sum2_size_sweep.py VARIANT_SET=focus)
# under two XCD stripe sizes (TIPS_STRIPE_KIB, read once per process), fresh processes, interleaved
# rounds. Output: gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-sum2_focus}"
mkdir -p "$OUT"
for r in ${ROUNDS_AB:-1 2 3}; do
  for k in ${STRIPES:-1024 512}; do
    echo "[$(date +%T)] round $r stripe $k" >> "$OUT/steps.txt"
    TIPS_STRIPE_KIB=$k VARIANT_SET=focus SIZES_MIB=${SIZES_MIB:-256,128} ROUNDS=7 timeout -k 10 200 \
      python3 tools/sum2_size_sweep.py > "$OUT/focus_s${k}_r$r.jsonl" 2> "$OUT/focus_s${k}_r$r.err" || exit 1
  done
done
echo "[$(date +%T)] done" >> "$OUT/steps.txt"
