#!/bin/bash
# Round-2 profiles of bench.py N=1 (config 2): rocprofv3 kernel-trace stats of the bench command,
# then the FETCH_SIZE / WRITE_SIZE PMC passes (tools/gpu_pmc.sh), each pass its own run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r02prof}"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ktrace" -o bench \
  -- python3 bench.py --no-cpu-baseline > "$OUT/ktrace.log" 2>&1 || exit $?
TAG=${TAG:-r02prof} bash tools/gpu_pmc.sh
