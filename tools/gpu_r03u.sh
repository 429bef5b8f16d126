#!/bin/bash
# r03u: the small host-call breakdown, and the op-body tests on the latest negotiation build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03u"
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/host_call_probe.py > "$OUT/host_call_probe.jsonl" 2> "$OUT/host_call_probe.err" || exit $?
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 250 --timeout-method thread tests/test_gpu_op_body.py tests/test_negotiation_cpu.py > "$OUT/pytest_op_body.log" 2>&1
