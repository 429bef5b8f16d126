#!/bin/bash
# r03p: where the box's host side is (NUMA) and the fused host path with the copy pool's threads
# bound to the GPU's node or not (tools/numa_probe.py), plus the same bytes as one host buffer.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03p"
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/numa_probe.py > "$OUT/numa_probe.jsonl" 2> "$OUT/numa_probe.err"
