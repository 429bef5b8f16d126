#!/bin/bash
# The direct schedule's fold at config 3's sub-chunk shape (8 x 32 MiB -> 32 MiB, 4 rotating sets,
# tools/multi_sum_pmc.py): FETCH_SIZE / WRITE_SIZE passes (each its own run) summarised as HBM bytes
# per launch (tools/pmc_traffic.py), then a kernel trace (--kernel-trace --stats) of
# tools/multi_sum_rate.py for the per-launch duration beside the events' rate.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-pmc_multi}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o multi \
    -- python3 tools/multi_sum_pmc.py > "$OUT/pmc_$c.log" 2>&1 || exit $?
done
python3 tools/pmc_traffic.py "$OUT/pmc_multi.json" --fetch "$OUT/pmc_FETCH_SIZE" --write "$OUT/pmc_WRITE_SIZE" \
  --kernel multi_sum --algo-bytes $((9 * 32 * 1024 * 1024)) \
  --note "direct fold, 8 x 32 MiB sources -> 32 MiB, 4 rotating buffer sets (tools/multi_sum_pmc.py)" > /dev/null || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o rate \
  -- python3 tools/multi_sum_rate.py > "$OUT/rate.jsonl" 2> "$OUT/rate.err" || exit $?
exit 0
