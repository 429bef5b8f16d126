#!/bin/bash
# The op-body C host over 3 RCCL ranks (96 tensors), run up to RUNS times, stopping at the first run
# that fails: every rank's stdout and stderr kept (the watchdog's state reports at 60 / 120 / 200 s
# say what the library's threads were doing). Each rank under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-hunt}"
mkdir -p "$OUT"
for ((k = 1; k <= ${RUNS:-5}; k++)); do
  port=$((30000 + RANDOM % 2000)) pids=() rc=0
  for r in 0 1 2; do
    RANK=$r WORLD_SIZE=3 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port TIPS_BOOTSTRAP_PORT=$port \
      NCCL_HOSTID=tips-hunt-$r NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 OP_BODY_TENSORS=96 \
      timeout -k 5 230 tools/_bin/${BIN:-op_body} > "$OUT/run${k}_r$r.out" 2> "$OUT/run${k}_r$r.err" &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait "$p" || rc=$?; done
  echo "run $k rc=$rc $(date +%T)" >> "$OUT/steps.txt"
  [ $rc -ne 0 ] && exit 0
done
