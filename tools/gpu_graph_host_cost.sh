#!/bin/bash
# Host cost of one tips_allreduce call, eager vs replayed plan (TIPS_GRAPHS), through the C-ABI on
# /opt/rocm's runtime: tools/_bin/graph_repro's timing loop (TIPS_REPRO_TIME calls of a 4099-float
# bucket) for p RCCL ranks sharing the GPU over the socket transport. One JSON line per rank and
# setting into gpurun_out/graph_host_cost.jsonl. enqueue_us is the host time inside tips_allreduce;
# call_us the wall time per call (socket-bound here, not xGMI).
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/graph_host_cost.jsonl
: > $OUT
export NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 TIPS_REPRO_TIME=${TIPS_REPRO_TIME:-400}
for cfg in "oneshot 2" "direct 3" "direct 4" "ring 4"; do
  set -- $cfg
  for g in 0 1; do
    rm -f /tmp/ghc_id
    pids=()
    for ((r = 0; r < $2; r++)); do
      TIPS_ALGO=$1 TIPS_GRAPHS=$g NCCL_HOSTID=ghc-$r timeout -k 10 180 tools/_bin/graph_repro $r $2 /tmp/ghc_id \
        | sed "s/^{/{\"algo\": \"$1\", \"graphs\": $g, /" >> $OUT &
      pids+=($!)
    done
    for p in "${pids[@]}"; do wait $p; done
  done
done
cat $OUT
