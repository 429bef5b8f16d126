#!/bin/bash
# Two ranks of tools/graph_repro sharing the GPU over RCCL's socket transport (NCCL_HOSTID per process).
cd "$(dirname "$0")/.."
export NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 TIPS_ALGO=${TIPS_ALGO:-oneshot}
rm -f /tmp/gr_id
NCCL_HOSTID=gr-0 timeout -k 10 120 tools/_bin/graph_repro 0 2 /tmp/gr_id &
a=$!
NCCL_HOSTID=gr-1 timeout -k 10 120 tools/_bin/graph_repro 1 2 /tmp/gr_id &
b=$!
wait $a; ra=$?
wait $b; rb=$?
echo "exit $ra $rb"
[ $ra -eq 0 ] && [ $rb -eq 0 ]
