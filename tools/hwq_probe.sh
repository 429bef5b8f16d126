#!/bin/bash
# Does the fused host path's H2D wait behind the D2H blits because their HIP streams share a hardware
# queue (GPU_MAX_HW_QUEUES, 4 by default)? config 5 host -> host (tools/host_fused_once.py) at 4, 8
# and 16 hardware queues, interleaved over 3 rounds, TIPS_HOST_TRACE=1. gpurun_out/$TAG/hwq.txt
set -e
OUT=gpurun_out/${TAG:-hwq}
mkdir -p "$OUT"
for round in 1 2 3; do
  for q in 4 8 16; do
    echo "== hwq $q" >> "$OUT/hwq.txt"
    GPU_MAX_HW_QUEUES=$q TIPS_HOST_TRACE=1 timeout -k 5 120 python tools/host_fused_once.py 4 2>&1 | grep -E "tips host|call ms" | tail -4 >> "$OUT/hwq.txt"
  done
done
