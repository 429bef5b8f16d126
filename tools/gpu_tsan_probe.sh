#!/bin/bash
# The op-body C host on the ThreadSanitizer build (tools/_bin/op_body_tsan), run by hand so each
# rank's sanitizer output is kept: one rank alone, then 2 RCCL ranks; every rank under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-tsan}"
mkdir -p "$OUT"
export TSAN_OPTIONS="halt_on_error=1 exitcode=66 report_signal_unsafe=0 suppressions=$PWD/tools/tsan.supp ${TSAN_EXTRA:-}"
run_ranks() {  # p tensors tag limit
  local p=$1 n=$2 tag=$3 lim=$4 port=$((29500 + RANDOM % 2000)) pids=() r rc=0
  for ((r = 0; r < p; r++)); do
    RANK=$r WORLD_SIZE=$p LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port TIPS_BOOTSTRAP_PORT=$port \
      NCCL_HOSTID=tips-tsan-$r NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 OP_BODY_TENSORS=$n \
      timeout -k 5 "$lim" tools/_bin/op_body_tsan > "$OUT/${tag}_r$r.out" 2> "$OUT/${tag}_r$r.err" &
    pids+=($!)
  done
  for r in "${!pids[@]}"; do wait "${pids[$r]}" || rc=$?; echo "$tag rank $r done rc=$rc" >> "$OUT/steps.txt"; done
  return $rc
}
run_ranks 1 8 one 60 || exit $?
run_ranks 2 16 two 120
