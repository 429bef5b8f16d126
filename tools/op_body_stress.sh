#!/bin/bash
# tools/_bin/op_body(_tsan) over 3 RCCL ranks on the box's GPU with more tensors and steps than the
# test (OP_BODY_TENSORS, OP_BODY_PASSES); BIN=op_body_tsan runs it under ThreadSanitizer.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-opbody_stress}
mkdir -p "$OUT"
BIN=${BIN:-op_body}
PORT=$((20000 + RANDOM % 20000))
export TSAN_OPTIONS="halt_on_error=1 exitcode=66 report_signal_unsafe=0 suppressions=$PWD/tools/tsan.supp"
for r in 0 1 2; do
  RANK=$r WORLD_SIZE=3 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT TIPS_BOOTSTRAP_PORT=$PORT \
    NCCL_HOSTID=tips-op-body-$r NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 OP_BODY_TENSORS=${TENSORS:-160} \
    OP_BODY_PASSES=${PASSES:-4} timeout -k 5 230 tools/_bin/$BIN > "$OUT/r$r.out" 2> "$OUT/r$r.err" &
done
rc=0
for j in $(jobs -p); do wait "$j" || rc=$?; done
tail -n1 "$OUT"/r*.out
exit $rc
