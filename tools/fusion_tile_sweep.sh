#!/bin/bash
# Fusion pack/unpack tile size sweep (configs 4 and 5 at one rank: the pack + unpack cost).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-tiles}
mkdir -p "$OUT"
for t in ${TILES:-65536 32768 16384 8192 4096}; do
  for w in fused1000 resnet50; do
    TIPS_COPY_TILE_BYTES=$t timeout -k 10 200 python bench.py --workload $w --no-compare --steps 50 \
      > "$OUT/${w}_$t.log" 2>&1 || exit $?
  done
done
