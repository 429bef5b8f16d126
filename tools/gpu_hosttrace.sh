#!/bin/bash
# HIP API trace of the N=1 fused1000 bench: what the host spends per fused call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-hosttrace}"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$OUT/f" -o trace \
  -- python3 bench.py --workload fused1000 --no-compare --steps 10 --warmup 3 > "$OUT/f.log" 2>&1 || exit $?
exit 0
