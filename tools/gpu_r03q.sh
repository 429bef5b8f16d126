#!/bin/bash
# r03q: host path + fused-copy tiles-per-workgroup sweep. Each GPU step under its own limit; stop at the
# first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03q"
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
step() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> "$OUT/steps.txt"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> "$OUT/steps.txt"; return $rc; }
step pytest_host 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_allreduce.py -k "host or fused" || exit 1
TIPS_COPY_TILES_PER_WG=4 step pytest_fused_pw4 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_allreduce.py -k "fused and not host" || exit 1
TIPS_HOST_TRACE=1 step probe 200 python -u tools/host_probe.py || exit 1
for pw in 1 2 4 8; do
  for w in fused1000 resnet50; do
    TIPS_COPY_TILES_PER_WG=$pw step "bench_${w}_pw$pw" 240 python -u bench.py --workload $w --no-compare || exit 1
  done
done
exit 0
