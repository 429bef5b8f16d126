#!/bin/bash
# tips_enqueue_allreduce_n: all of a list's requests committed under one lock hold (TIPS_LIST_ONE_LOCK=1,
# shipped) or one commit each (0, round 3's behaviour), 1000 named device requests (bench.py --workload
# negotiated1000), interleaved over 4 rounds. gpurun_out/$TAG/list_ab.jsonl
set -e
OUT=gpurun_out/${TAG:-listab}
mkdir -p "$OUT"
for round in 1 2 3 4; do
  for v in 0 1; do
    printf '== one_lock %s ' "$v" >> "$OUT/list_ab.jsonl"
    TIPS_LIST_ONE_LOCK=$v timeout -k 5 120 python bench.py --workload negotiated1000 --no-sub --no-cpu-baseline 2>/dev/null \
      | grep '^{' >> "$OUT/list_ab.jsonl"
  done
done
