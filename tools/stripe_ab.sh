#!/bin/bash
# A/B of the XCD stripe map (TIPS_STRIPE_KIB: 0 = contiguous eighths per XCD, 1024 = 1 MiB stripes,
# the default) on the kernels that use it, interleaved rounds, each run a fresh process (the
# setting is read once): the headline (config 2, sum2_buf_kernel), config 3 at one rank
# (copy_buf_kernel, 1 GiB), and the direct schedule's fold at 8 x 32 / 8 x 8 / 4 x 64 / 2 x 128 MiB
# (multi_sum_buf_kernel, tools/multi_sum_rate.py). Output: gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-stripe_ab}"
mkdir -p "$OUT"
for r in ${ROUNDS:-1 2}; do
  for k in ${STRIPES:-0 1024}; do
    echo "[$(date +%T)] round $r stripe $k" >> "$OUT/steps.txt"
    TIPS_STRIPE_KIB=$k timeout -k 10 120 python3 bench.py --no-sub --no-cpu-baseline --no-extras --steps 200 --warmup 20 \
      > "$OUT/config2_s${k}_r$r.jsonl" 2> "$OUT/config2_s${k}_r$r.err" || exit 1
    TIPS_STRIPE_KIB=$k timeout -k 10 120 python3 bench.py --workload bucket --no-sub --no-cpu-baseline --steps 20 --warmup 3 \
      > "$OUT/bucket_s${k}_r$r.jsonl" 2> "$OUT/bucket_s${k}_r$r.err" || exit 1
    TIPS_STRIPE_KIB=$k timeout -k 10 120 python3 tools/multi_sum_rate.py > "$OUT/fold_s${k}_r$r.jsonl" \
      2> "$OUT/fold_s${k}_r$r.err" || exit 1
  done
done
echo "[$(date +%T)] done" >> "$OUT/steps.txt"
