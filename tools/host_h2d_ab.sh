#!/bin/bash
# the fused host path's H2D by the DMA engine (hipMemcpyAsync) or by copy_buf_kernel reading the
# page-locked slot (TIPS_HOST_H2D_KERNEL=1), config 5 host -> host, flat (tools/host_fused_once.py)
# and through named requests (tools/_bin/op_host), interleaved over 3 rounds. gpurun_out/$TAG/h2d_ab.txt
set -e
OUT=gpurun_out/${TAG:-h2dab}
mkdir -p "$OUT"
for round in 1 2 3; do
  for k in 0 1; do
    echo "== h2d_kernel $k" >> "$OUT/h2d_ab.txt"
    TIPS_HOST_H2D_KERNEL=$k TIPS_HOST_TRACE=1 timeout -k 5 120 python tools/host_fused_once.py 4 2>&1 | grep -E "tips host|call ms" | tail -4 >> "$OUT/h2d_ab.txt"
    TIPS_HOST_H2D_KERNEL=$k OP_HOST_STEPS=15 timeout -k 5 60 tools/_bin/op_host >> "$OUT/h2d_ab.txt" 2>&1
  done
done
