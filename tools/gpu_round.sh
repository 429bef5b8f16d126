#!/bin/bash
# Runs on the GPU box (via gpurun): parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash / abort / timeout ends the script
# (test FAILURES, exit 1, do not: the bench still runs so the numbers are recorded).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-round}"
mkdir -p "$OUT"
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

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  if [ -n "${PYTEST_K:-}" ]; then
    run pytest_gpu "${PYTEST_TIMEOUT:-1100}" python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread -k "$PYTEST_K"
  else
    run pytest_gpu "${PYTEST_TIMEOUT:-1100}" python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread
  fi
  rc=$?; fatal $rc && exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  rc=$?; fatal $rc && exit $rc
fi
run bench 600 python bench.py ${BENCH_ARGS:-}
rc=$?; fatal $rc && exit $rc
if [ "${EXTRA:-1}" = "1" ]; then
  for w in ${WORKLOADS:-bucket fused1000 resnet50 negotiated1000}; do
    run bench_$w 300 python bench.py --workload $w --no-compare
    rc=$?; fatal $rc && exit $rc
  done
fi
if [ "${CPU_SWEEP:-0}" = "1" ]; then  # host cores only: the reference's MPI path and c = a + b
  run cpu_ref_sweep 900 python tools/cpu_ref_sweep.py
  rc=$?; fatal $rc && exit $rc
fi
if [ "${PROFILE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  run rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_stats" -o bench \
      -- python3 bench.py --no-cpu-baseline --no-extras ${BENCH_ARGS:-}
  rc=$?; fatal $rc && exit $rc
fi
exit 0
