#!/bin/bash
# Does the config-2 line depend on how long the GPU has been busy before the timed launches?
# Fresh processes, interleaved rounds: the driver-like short run (--steps 20 --warmup 5), the default
# (200 / 20) and a long warm-up (200 / 2000), all HBM-only over the 4 rotating triples.
# Output: gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-warmup_ab}"
mkdir -p "$OUT"
for r in ${ROUNDS:-1 2 3}; do
  for sw in 20:5 200:20 200:2000; do
    s=${sw%%:*} w=${sw##*:}
    echo "[$(date +%T)] round $r steps $s warmup $w" >> "$OUT/steps.txt"
    timeout -k 10 120 python3 bench.py --no-sub --no-cpu-baseline --no-extras --steps $s --warmup $w \
      > "$OUT/b_s${s}_w${w}_r$r.jsonl" 2> "$OUT/b_s${s}_w${w}_r$r.err" || exit 1
  done
done
echo "[$(date +%T)] done" >> "$OUT/steps.txt"
