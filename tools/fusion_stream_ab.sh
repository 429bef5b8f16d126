#!/bin/bash
# the one-rank fused step (configs 4 and 5, TIPS_FUSION_MEASURE_PACK as bench.py sets it) with the
# pack / unpack kernels on the caller's stream in one event chain (TIPS_FUSION_CALLER_STREAM=1,
# shipped) or on the library's fusion stream joined with the caller (0, round 3), interleaved over
# 3 rounds. gpurun_out/$TAG/fusion_stream_ab.txt
set -e
OUT=gpurun_out/${TAG:-fusionstream}
mkdir -p "$OUT"
for round in 1 2 3; do
  for w in fused1000 resnet50; do
    for v in 0 1; do
      printf '== %s caller_stream %s ' "$w" "$v" >> "$OUT/fusion_stream_ab.txt"
      TIPS_FUSION_CALLER_STREAM=$v timeout -k 5 120 python bench.py --workload $w --no-sub --no-cpu-baseline 2>/dev/null \
        | grep '^{' >> "$OUT/fusion_stream_ab.txt"
    done
  done
done
