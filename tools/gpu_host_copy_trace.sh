#!/bin/bash
# The fused host path's DMA copies, one by one: rocprofv3 memory-copy + kernel trace of
# tools/host_fused_once.py (no counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r03c}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for p in ${PIECES:-8388608}; do
  TIPS_HOST_FUSED_PIECE_BYTES=$p TIPS_HOST_TRACE=${TIPS_HOST_TRACE:-1} timeout -k 10 180 rocprofv3 --memory-copy-trace --kernel-trace \
      --output-format csv -d "$OUT/copytrace_$p" -o run -- python3 tools/host_fused_once.py 4 \
      > "$OUT/copytrace_$p.log" 2>&1 || exit $?
done
