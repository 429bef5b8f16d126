#!/bin/bash
# Round-2 GPU pass (via gpurun): full -m gpu suite, smoke, the N=1 bench lines, and N>1 rehearsals
# of bench.py over real RCCL ranks sharing the one GPU (TIPS_BENCH_FAKE_HOSTS=1: socket transport,
# so their rates are not xGMI rates). Every GPU step has its own time limit; a crash / timeout ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r02}"
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
# a heartbeat under gpurun_out: a multi-process test that runs for minutes prints nothing meanwhile
# (each step keeps its own time limit, so a real hang still ends)
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
trap 'kill $! 2>/dev/null' EXIT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  run pytest_gpu "${PYTEST_TIMEOUT:-1100}" python -u -m pytest tests -v -m gpu --timeout 600 --timeout-method thread ${PYTEST_ARGS:-}
  rc=$?; fatal $rc && exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  rc=$?; fatal $rc && exit $rc
fi
run bench_n1 300 python -u bench.py; rc=$?; fatal $rc && exit $rc
run bench_n1_fused1000 300 python -u bench.py --workload fused1000; rc=$?; fatal $rc && exit $rc
run bench_n1_resnet50 300 python -u bench.py --workload resnet50; rc=$?; fatal $rc && exit $rc
if [ "${REHEARSE:-1}" = "1" ]; then
  TIPS_BENCH_FAKE_HOSTS=1 run rehearsal_n2 400 python -u bench.py --gpus 2 --bucket-mib 64 --steps 3 --warmup 1
  rc=$?; fatal $rc && exit $rc
  TIPS_BENCH_FAKE_HOSTS=1 run rehearsal_n4_resnet50 500 python -u bench.py --gpus 4 --workload resnet50 --steps 3 --warmup 1
  rc=$?; fatal $rc && exit $rc
fi
exit 0
