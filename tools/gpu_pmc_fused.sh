#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE: one counter per run) over bench.py's one-rank fused lines
# (configs 4 and 5), for the fusion pack kernel's HBM bytes per launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-pmcfused}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in fused1000 resnet50; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/${w}_$c" -o bench \
      -- python3 bench.py --workload $w --steps 20 --warmup 2 > "$OUT/${w}_$c.log" 2>&1 || exit $?
  done
done
exit 0
