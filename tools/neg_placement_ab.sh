#!/bin/bash
# is the negotiated path's bimodality (0.40 vs 0.87-1.85 us per tensor for 1000
# named requests at one rank) a matter of where its threads run? ROUNDS rounds, each running
# bench.py --workload negotiated1000 once per TIPS_NEG_BIND setting in a fresh process (settings
# interleaved, order alternating); every line carries per_tensor_us and the threads' placement
# (configs... .placement: CPU, L3 domain, socket of the caller, tips-neg, tips-done).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-negplace}"
mkdir -p "$OUT"
SETTINGS=${SETTINGS:-"none l3"}
for r in $(seq 1 "${ROUNDS:-4}"); do
  order=$SETTINGS
  [ $((r % 2)) -eq 0 ] && order=$(echo "$SETTINGS" | tr ' ' '\n' | tac | tr '\n' ' ')
  for b in $order; do
    bind=$b; [ "$b" = none ] && bind=0
    echo "[$(date +%T)] round $r bind=$b" >> "$OUT/steps.txt"
    TIPS_NEG_BIND=$bind timeout -k 10 120 python3 bench.py --workload negotiated1000 --no-cpu-baseline --steps 20 \
      --warmup 5 > "$OUT/r${r}_${b}.jsonl" 2> "$OUT/r${r}_${b}.err" || { echo "rc=$?" >> "$OUT/steps.txt"; exit 1; }
  done
done
