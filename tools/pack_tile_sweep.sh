#!/bin/bash
# the fusion pack kernel (copy_segs_kernel) per bucket launch at 4 / 8 / 16 KiB tiles
# (TIPS_COPY_TILE_BYTES), configs 4 and 5, their own layouts and a contiguous tensor of the same
# size, interleaved over 3 rounds of tools/pack_ceiling.py. gpurun_out/$TAG/pack_tile_sweep.txt
set -e
OUT=gpurun_out/${TAG:-packtile}
mkdir -p "$OUT"
for round in 1 2 3; do
  for t in 4096 8192 16384; do
    TIPS_COPY_TILE_BYTES=$t timeout -k 5 120 python tools/pack_ceiling.py 5 --only=config4/pack --only=config5/pack \
      --only=config4/contig --only=config5/contig 2>/dev/null | sed "s/^/tile $t /" >> "$OUT/pack_tile_sweep.txt"
  done
done
