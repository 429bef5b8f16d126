#!/bin/bash
# The TF-op-shaped host path (tools/op_host.c: config 5 as 214 named host requests from 4 executor
# threads) under each TIPS_NEG_BIND setting, interleaved over ROUNDS rounds, beside the single fused
# host call (tools/host_fused_once.py). Each op_host line carries the placement of its main thread and
# the library's threads (name:cpu/first CPU of the L3/socket). Results in gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-opbind}
mkdir -p "$OUT"
export MASTER_ADDR=127.0.0.1
OP_HOST_STEPS=5 MASTER_PORT=29590 timeout -k 5 60 tools/_bin/op_host > "$OUT/first_run.txt" 2>&1 || true
for round in $(seq 1 "${ROUNDS:-3}"); do
  for b in ${SETTINGS:-0 l3 core}; do
    printf '%s ' "bind=$b" >> "$OUT/sweep.txt"
    TIPS_NEG_BIND=$b MASTER_PORT=$((29600 + RANDOM % 200)) OP_HOST_THREADS=4 OP_HOST_STEPS=20 timeout -k 5 60 \
      tools/_bin/op_host >> "$OUT/sweep.txt" 2>&1 || { echo "rc=$?" >> "$OUT/sweep.txt"; exit 1; }
  done
  printf 'fused ' >> "$OUT/sweep.txt"
  timeout -k 5 120 python3 tools/host_fused_once.py >> "$OUT/sweep.txt" 2>&1 || exit 1
done
