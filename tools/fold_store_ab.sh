#!/bin/bash
# A/B of the capped fold's store policy (TIPS_FOLD_STORE: sc1, the default, or nt; read once per
# process) under the XCD stripe map: the fold tests under nt stores (bit-exact), then
# tools/multi_sum_rate.py in fresh processes, interleaved rounds. Output: gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-fold_store_ab}"
mkdir -p "$OUT"
TIPS_FOLD_STORE=nt timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -q -m gpu --timeout 120 \
  --timeout-method thread -k "multi or fold" > "$OUT/pytest.txt" 2>&1 || exit 1
for r in ${ROUNDS:-1 2 3}; do
  for k in sc1 nt; do
    echo "[$(date +%T)] round $r store $k" >> "$OUT/steps.txt"
    TIPS_FOLD_STORE=$k timeout -k 10 120 python3 tools/multi_sum_rate.py > "$OUT/fold_${k}_r$r.jsonl" \
      2> "$OUT/fold_${k}_r$r.err" || exit 1
  done
done
echo "[$(date +%T)] done" >> "$OUT/steps.txt"
