#!/bin/bash
# Round-3 PMC passes (FETCH_SIZE, WRITE_SIZE: one counter per run, no traces): the bucket-sum kernel
# under bench.py's default command, and the fusion pack kernel's per-bucket launches of configs 4
# and 5 alone (tools/pack_ceiling.py --only=configN/pack); then the kernel-trace summary of the
# default bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r03pmc}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/sum_$c" -o run \
    -- python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 2 > "$OUT/sum_$c.log" 2>&1 || exit $?
  for w in config4 config5; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/${w}_$c" -o run \
      -- python3 tools/pack_ceiling.py 3 --only=$w/pack > "$OUT/${w}_$c.log" 2>&1 || exit $?
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_stats" -o bench \
    -- python3 bench.py --no-cpu-baseline --no-extras > "$OUT/prof_stats.log" 2>&1
