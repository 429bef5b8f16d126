#!/bin/bash
# A focused GPU pass (via gpurun) while iterating: the pytest node ids / -k expression in $TESTS,
# then optional bench lines ($BENCH: space-separated workloads, "-" for none). Every GPU step has
# its own time limit; a crash or timeout ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-quick}"
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS="$OUT/steps.txt"
: > "$STEPS"
run() {  # name seconds cmd...
  local name=$1 t=$2
  shift 2
  echo "[$(date +%T)] start $name" >> "$STEPS"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$STEPS"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
if [ -n "${TESTS:-}" ]; then
  # shellcheck disable=SC2086
  run pytest "${PYTEST_TIMEOUT:-900}" python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread $TESTS ${KEXPR:+-k "$KEXPR"}
  rc=$?; fatal $rc && exit $rc
fi
for w in ${BENCH:--}; do
  [ "$w" = "-" ] && continue
  run "bench_$w" 300 python -u bench.py --workload "$w" ${BENCH_ARGS:-}
  rc=$?; fatal $rc && exit $rc
done
exit 0
