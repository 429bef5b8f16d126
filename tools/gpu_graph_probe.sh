#!/bin/bash
# Which HIP-graph capture patterns work with this ROCm / RCCL (tools/graph_probe.cc), one rank and
# two ranks sharing the GPU over RCCL's socket transport. Stops at the first failure.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
P=tools/_bin/graph_probe
[ -x $P ] || { echo "build $P first"; exit 2; }
for m in ${MODES1:-0 1 2 3 4}; do
  rm -f /tmp/gp_id
  timeout -k 10 60 $P 0 1 $m /tmp/gp_id
done
export NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1
for m in ${MODES2:-1 2 3 4}; do
  rm -f /tmp/gp_id
  NCCL_HOSTID=gp-0 timeout -k 10 90 $P 0 2 $m /tmp/gp_id &
  a=$!
  NCCL_HOSTID=gp-1 timeout -k 10 90 $P 1 2 $m /tmp/gp_id &
  b=$!
  wait $a
  wait $b
done
echo ALL_DONE
