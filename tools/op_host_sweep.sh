#!/bin/bash
# A/B of the named-request enqueue on one box (tools/op_host.c: config 5 as 214 named host requests):
# variants interleaved over 3 rounds, at 1 and 4 executor threads -
#   enqueue:  pointers classified in the enqueue, plain mutexes (round 3)
#   deferred: classified by the negotiation thread, plain mutexes
#   adaptive: classified by the negotiation thread, adaptive mutexes (shipped)
# then one traced run of the shipped variant. Results in gpurun_out/$TAG/.
set -e
OUT=gpurun_out/${TAG:-opsweep}
mkdir -p "$OUT"
run() {  # label threads env...
  local label=$1 t=$2
  shift 2
  printf '%s threads %s ' "$label" "$t" >> "$OUT/sweep.txt"
  env "$@" OP_HOST_THREADS=$t OP_HOST_STEPS=15 timeout -k 5 60 tools/_bin/op_host >> "$OUT/sweep.txt" 2>&1
}
for round in 1 2 3; do
  for t in 1 4; do
    run enqueue $t TIPS_CLASSIFY_AT_ENQUEUE=1 TIPS_ADAPTIVE_LOCKS=0
    run deferred $t TIPS_CLASSIFY_AT_ENQUEUE=0 TIPS_ADAPTIVE_LOCKS=0
    run adaptive $t TIPS_CLASSIFY_AT_ENQUEUE=0 TIPS_ADAPTIVE_LOCKS=1
  done
done
OP_HOST_TRACE=1 OP_HOST_THREADS=4 OP_HOST_STEPS=4 timeout -k 5 60 tools/_bin/op_host > "$OUT/trace_4.txt" 2>&1
