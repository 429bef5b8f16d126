#!/bin/bash
# Host copy threads (TIPS_HOST_THREADS) for the fused host call and the op path (tools/op_host.c),
# interleaved over 3 rounds on one box; one untimed op_host run first (fresh-box DMA warm-up).
set -e
OUT=gpurun_out/${TAG:-hostthreads}
mkdir -p "$OUT"
export MASTER_ADDR=127.0.0.1
OP_HOST_STEPS=5 MASTER_PORT=29590 timeout -k 5 60 tools/_bin/op_host > "$OUT/first_run.txt" 2>&1 || true
for round in 1 2 3; do
  for t in 8 12 16; do
    printf 'op_host threads %s ' $t >> "$OUT/sweep.txt"
    TIPS_HOST_THREADS=$t MASTER_PORT=$((29600 + RANDOM % 200)) OP_HOST_THREADS=4 OP_HOST_STEPS=20 \
      timeout -k 5 60 tools/_bin/op_host >> "$OUT/sweep.txt" 2>&1
    printf 'host_fused threads %s ' $t >> "$OUT/sweep.txt"
    TIPS_HOST_THREADS=$t timeout -k 5 120 python3 tools/host_fused_once.py 15 2>/dev/null | tail -15 | tr '\n' ' ' \
      >> "$OUT/sweep.txt"
    echo >> "$OUT/sweep.txt"
  done
done
