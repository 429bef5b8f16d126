#!/bin/bash
# r03s2: the FusedList change - fusion and grads GPU tests, then the fused bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03s2"
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_allreduce.py tests/test_gpu_rccl_procs.py -k "fus or flat or grads or pack or layout or list or optimizer" > "$OUT/pytest_fusion.log" 2>&1 || exit $?
for w in fused1000 resnet50; do
  timeout -k 10 240 python -u bench.py --workload $w --no-compare > "$OUT/bench_$w.log" 2>&1 || exit $?
done
