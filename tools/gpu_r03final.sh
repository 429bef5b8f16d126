#!/bin/bash
# r03final: the final tree once more (after the list-enqueue pointer cache and table reuse) on a fresh box - the whole GPU suite, smoke(), bench.py's default
# N = 1 line, and the negotiated-path line (after the batch-event change), each under its own
# limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r03final"
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
step() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> "$OUT/steps.txt"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> "$OUT/steps.txt"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread || exit 1
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
step bench_negotiated1000 240 python -u bench.py --workload negotiated1000 --no-compare || exit 1
step bench 600 python -u bench.py || exit 1
exit 0
