#!/bin/bash
# One GPU-box session: the steps named in STEPS, in order, each under its own time limit, stopping
# at the first failure (a GPU fault, abort or time limit ends the call: nothing more runs on the GPU).
# Everything lands in gpurun_out/$TAG/. Steps:
#   pytest      python -m pytest $PYTEST_ARGS (default: the whole -m gpu suite)
#   bench1      python bench.py (N = 1, the driver's default command)        -> bench_n1.jsonl
#   bench1prof  rocprofv3 --kernel-trace --stats of bench.py --no-sub          -> prof/
#   rehearse2   bench.py --gpus 2 over the socket transport (TIPS_BENCH_FAKE_HOSTS=1)  -> rehearsal_n2.log
#   rehearse4   the same at N = 4 (with its peer-schedule child jobs: 4 + 4 processes on the GPU)
#   rehearse8   the same at N = 8 (its child jobs would put 16+ processes on the one GPU: the box's
#               process guard allows 16, so run it with TIPS_BENCH_PEER_CHILD=0 or --no-env-variants)                                             -> rehearsal_n8.log
#   smoke       __graft_entry__.smoke()
#   custom      bash -c "$CUSTOM"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-check}"
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 30; do date +%T >> "$OUT/heartbeat.txt"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # name timeout cmd...
  local name=$1 t=$2
  shift 2
  echo "[$(date +%T)] $name start" >> "$OUT/steps.txt"
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$OUT/steps.txt"
  return $rc
}
for s in ${STEPS:-pytest bench1}; do
  case $s in
    pytest) run pytest "${PYTEST_TIMEOUT:-1100}" python -u -m pytest ${PYTEST_ARGS:-tests -m gpu} -x -q --timeout 300 \
              --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit $? ;;
    bench1) run bench1 "${BENCH_TIMEOUT:-500}" python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench_n1.jsonl" \
              2> "$OUT/bench_n1.err" || exit $? ;;
    bench1prof) run bench1prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py \
                  --no-sub --no-cpu-baseline --no-extras --steps 200 --warmup 20 > "$OUT/bench_prof.log" 2>&1 || exit $? ;;
    rehearse2) TIPS_BENCH_FAKE_HOSTS=1 run rehearse2 "${N2_TIMEOUT:-600}" python -u bench.py --gpus 2 ${REHEARSE_ARGS:-} \
                 > "$OUT/rehearsal_n2.log" 2>&1 || exit $? ;;
    rehearse4) TIPS_BENCH_FAKE_HOSTS=1 run rehearse4 "${N4_TIMEOUT:-700}" python -u bench.py --gpus 4 ${REHEARSE_ARGS:-} \
                 > "$OUT/rehearsal_n4.log" 2>&1 || exit $? ;;
    rehearse8) TIPS_BENCH_FAKE_HOSTS=1 run rehearse8 "${N8_TIMEOUT:-700}" python -u bench.py --gpus 8 ${REHEARSE_ARGS:-} \
                 > "$OUT/rehearsal_n8.log" 2>&1 || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $? ;;
    custom) run custom "${CUSTOM_TIMEOUT:-600}" bash -c "$CUSTOM" > "$OUT/custom.log" 2>&1 || exit $? ;;
    *) echo "unknown step $s" >> "$OUT/steps.txt"; exit 2 ;;
  esac
done
