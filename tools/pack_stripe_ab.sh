#!/bin/bash
# A/B of the fusion pack's workgroup -> slot map (TIPS_PACK_STRIPE_KIB: 0 = one contiguous eighth
# of the slots per XCD, the default; 512 / 1024 = stripes dealt round-robin over the 8 XCDs, the
# layout's boundary tiles placed by the same map). First the fusion GPU tests under 1 MiB stripes
# (bit-exact), then tools/pack_ceiling.py's per-bucket pack and one-contiguous-tensor launches for
# configs 4 and 5, interleaved rounds, each run a fresh process (the knob is read once).
# Output: gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-pack_stripe_ab}"
mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "[$(date +%T)] tests" >> "$OUT/steps.txt"
  TIPS_PACK_STRIPE_KIB=1024 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_allreduce.py -q -m gpu \
    --timeout 120 --timeout-method thread -k "fused or fusion" > "$OUT/pytest.txt" 2>&1 || exit 1
fi
for r in ${ROUNDS:-1 2}; do
  for ko in ${STRIPES:-0:2 1024:2 512:2}; do  # stripe KiB : TIPS_COPY_ORDER (2 = boundary tiles spread, 0 = address order)
    k=${ko%%:*} o=${ko##*:}
    echo "[$(date +%T)] round $r stripe $k order $o" >> "$OUT/steps.txt"
    TIPS_COPY_ORDER=$o TIPS_PACK_STRIPE_KIB=$k timeout -k 10 180 python3 tools/pack_ceiling.py 3 --only=config4/pack --only=config4/contig_b0 \
      --only=config5/pack --only=config5/contig_b0 > "$OUT/pack_s${k}_o${o}_r$r.jsonl" 2> "$OUT/pack_s${k}_o${o}_r$r.err" || exit 1
  done
done
echo "[$(date +%T)] done" >> "$OUT/steps.txt"
