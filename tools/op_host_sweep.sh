#!/bin/bash
# A/B of the TF-op-shaped host path on one box (tools/op_host.c: config 5 as 214 named host requests
# from 4 executor threads), variants interleaved over 3 rounds:
#   one_call: tips_enqueue_allreduce_cb (request + callback in one call; shipped op body, round 5)
#   one_call_noexpect: without the linger's early end once the previous batch is complete
#     (TIPS_LINGER_EXPECT=0)
#   one_call_slack50: that, with Linux's default 50 us timer slack on the negotiation thread
#   one_call_locked: that and round 4's locked commit (TIPS_ENQUEUE_LOCKFREE=0)
#   two_call: tips_enqueue_allreduce_shaped + tips_on_done (round 4's op body)
# (round 5's earlier variants, e.g. TIPS_LINGER_SPIN=1: profiles/r05/aa_op_host_ab.txt)
# beside the single fused host call the ratio is taken against (tools/host_fused_once.py, the
# body of bench.py's host_to_host_fused), then one traced run of each. Results in gpurun_out/$TAG/.
set -e
OUT=gpurun_out/${TAG:-opsweep}
mkdir -p "$OUT"
export MASTER_ADDR=127.0.0.1
# (the first op_host process on a fresh box ran every step's H2D at 23 GiB/s against 36 for the
# next ones, profiles/r05/z_op_host_first_process.txt: one untimed run first)
OP_HOST_STEPS=5 MASTER_PORT=29590 timeout -k 5 60 tools/_bin/op_host > "$OUT/first_run.txt" 2>&1 || true
run() {  # label env...
  local label=$1
  shift 1
  printf '%s ' "$label" >> "$OUT/sweep.txt"
  env "$@" MASTER_PORT=$((29600 + RANDOM % 200)) OP_HOST_THREADS=4 OP_HOST_STEPS=20 timeout -k 5 60 tools/_bin/op_host \
    >> "$OUT/sweep.txt" 2>&1
}
for round in 1 2 3; do
  run one_call OP_HOST_ONE_CALL=1
  run one_call_noexpect OP_HOST_ONE_CALL=1 TIPS_LINGER_EXPECT=0
  run one_call_slack50 OP_HOST_ONE_CALL=1 TIPS_LINGER_EXPECT=0 TIPS_NEG_TIMER_SLACK_NS=50000
  run one_call_locked OP_HOST_ONE_CALL=1 TIPS_LINGER_EXPECT=0 TIPS_ENQUEUE_LOCKFREE=0 TIPS_NEG_TIMER_SLACK_NS=50000
  run two_call OP_HOST_ONE_CALL=0
  printf 'host_fused ' >> "$OUT/sweep.txt"
  timeout -k 5 120 python3 tools/host_fused_once.py 15 2>/dev/null | tail -15 | tr '\n' ' ' >> "$OUT/sweep.txt"
  echo >> "$OUT/sweep.txt"
done
for v in 1 0; do
  TIPS_LINGER_EXPECT=$v OP_HOST_TRACE=1 TIPS_NEG_TRACE=1 MASTER_PORT=$((29800 + v)) OP_HOST_THREADS=4 OP_HOST_STEPS=6 \
    timeout -k 5 60 tools/_bin/op_host > "$OUT/trace_expect_$v.txt" 2>&1
done
