#!/bin/bash
# r03r: host path with streaming-store host copies vs without; fused host tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03r"
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
step() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> "$OUT/steps.txt"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> "$OUT/steps.txt"; return $rc; }
step pytest_host 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_allreduce.py -k "host" || exit 1
for k in 1 2; do
  TIPS_HOST_TRACE=1 step "probe_stream_$k" 200 python -u tools/host_probe.py || exit 1
  TIPS_HOST_STREAM_STORES=0 TIPS_HOST_TRACE=1 step "probe_nostream_$k" 200 python -u tools/host_probe.py || exit 1
done
step bench_resnet50 240 python -u bench.py --workload resnet50 --no-compare || exit 1
exit 0
