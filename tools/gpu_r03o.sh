#!/bin/bash
# r03o: boundary tiles first in the pack kernel (TIPS_COPY_ORDER) - the fusion tests, then the
# per-bucket pack launches of configs 4 and 5 in tile order (0) and boundary-first order (1),
# alternating processes, and the fused bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03o"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_allreduce.py tests/test_gpu_rccl_procs.py -k "fus or flat or grads or pack or layout" > "$OUT/pytest_fusion.log" 2>&1 || exit $?
for k in 1 2 3; do
  for o in 0 1; do
    TIPS_COPY_ORDER=$o timeout -k 10 120 python -u tools/pack_ceiling.py 5 --only=config4/pack --only=config5/pack > "$OUT/order${o}_$k.jsonl" 2> "$OUT/order${o}_$k.err" || exit $?
  done
done
for w in fused1000 resnet50; do
  timeout -k 10 240 python -u bench.py --workload $w --no-compare > "$OUT/bench_$w.log" 2>&1 || exit $?
done
