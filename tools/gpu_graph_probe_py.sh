#!/bin/bash
# tools/graph_probe.py's capture patterns on torch's bundled HIP / RCCL: one rank, then two ranks
# sharing the GPU over RCCL's socket transport. Stops at the first failure.
set -e
cd "$(dirname "$0")/.."
for m in ${MODES1:-1 2 3 4}; do
  rm -f /tmp/gpp_id
  timeout -k 10 120 python tools/graph_probe.py 0 1 $m /tmp/gpp_id
done
export NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1
for m in ${MODES2:-1 2 3 4}; do
  rm -f /tmp/gpp_id
  NCCL_HOSTID=gpp-0 timeout -k 10 120 python tools/graph_probe.py 0 2 $m /tmp/gpp_id &
  a=$!
  NCCL_HOSTID=gpp-1 timeout -k 10 120 python tools/graph_probe.py 1 2 $m /tmp/gpp_id &
  b=$!
  wait $a
  wait $b
done
echo ALL_DONE
