#!/bin/bash
# r03q2: the host output pool - numa probe (one host buffer of config 5's bytes, fused lists) and
# the resnet50 bench line (per-tensor host path), plus the host tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03q2"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 150 --timeout-method thread tests/test_gpu_allreduce.py tests/test_gpu_rccl_procs.py -k "host" > "$OUT/pytest_host.log" 2>&1 || exit $?
timeout -k 10 300 python -u tools/numa_probe.py > "$OUT/numa_probe.jsonl" 2> "$OUT/numa_probe.err" || exit $?
timeout -k 10 240 python -u bench.py --workload resnet50 --no-compare > "$OUT/bench_resnet50.log" 2>&1
