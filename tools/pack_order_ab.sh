#!/bin/bash
# config 4's fusion pack (copy_segs_kernel) per bucket launch at 8 and 16 KiB tiles, with the
# layout's boundary tiles first (TIPS_COPY_ORDER=1), first within each XCD's share (2) and in address
# order (0), interleaved
# over 2 rounds of tools/pack_ceiling.py. gpurun_out/$TAG/pack_order_ab.txt
set -e
OUT=gpurun_out/${TAG:-packorder}
mkdir -p "$OUT"
for round in 1 2; do
  for t in ${TILES:-8192 16384}; do
    for o in ${ORDERS:-1 2 0}; do
      TIPS_COPY_TILE_BYTES=$t TIPS_COPY_ORDER=$o timeout -k 5 120 python tools/pack_ceiling.py 5 \
        --only=config4/pack --only=config5/pack 2>/dev/null | sed "s/^/tile $t order $o /" >> "$OUT/pack_order_ab.txt"
    done
  done
done
