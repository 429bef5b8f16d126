#!/bin/bash
# Kernel trace of the N=1 fused bench lines (where does a fused step's time go?)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-fusedprof}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in fused1000 resnet50; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$w" -o trace \
    -- python3 bench.py --workload $w --no-compare --steps 20 --warmup 3 > "$OUT/$w.log" 2>&1 || exit $?
done
timeout -k 10 300 python3 tools/copy_sweep.py 3 > "$OUT/copy_sweep.jsonl" 2> "$OUT/copy_sweep.err" || exit $?
exit 0
