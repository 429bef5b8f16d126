#!/bin/bash
# bench.py --workload negotiated1000 (config 4 as 1000 named requests, one rank) under a few
# negotiation settings, each in its own process with TIPS_NEG_TRACE=1; results in gpurun_out/$TAG/.
set -u
OUT=gpurun_out/${TAG:-negab}
mkdir -p "$OUT"
i=0
for v in ${VARIANTS:-base TIPS_RESPONSE_CACHE=0 TIPS_LINGER_EXPECT=0 TIPS_GRAPHS=0 base}; do
  i=$((i + 1))
  if [ "$v" = base ]; then set -- ; else set -- "$v"; fi
  env "$@" TIPS_NEG_TRACE=${TRACE:-1} timeout -k 10 100 python3 -u bench.py --workload negotiated1000 --no-cpu-baseline \
    --steps 10 --warmup 3 > "$OUT/run$i.json" 2> "$OUT/run$i.err" || exit 1
  printf '%s %s\n' "$v" "$(grep '^{' "$OUT/run$i.json" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["host_us_per_tensor"])')" >> "$OUT/res.txt"
done
