#!/bin/bash
# The capture experiments of DESIGN §4 (round 6), in order, each under its own time limit, stopping at
# the first failure (a crash ends the call). EXP names the steps; results in gpurun_out/$TAG/.
#   hip_<mode>      tools/_bin/capture_race_hip <mode>: the runtime alone (no RCCL, no library)
#   hipmode_<churn>_<capture mode>   the same with relaxed | thread | global capture
#   lib_<mode>      tools/_bin/capture_race over 2 RCCL ranks, churn <mode>, replays at their default (off)
#   libg_<mode>     the same with replays on (TIPS_GRAPHS=1)
#   opbody_nb_neg   op_body over 3 ranks, captures allowed on the negotiation thread, non-blocking threads
#   opbody_neg      the same with the threads' legacy-stream calls (the round-5 failure)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-race}"
mkdir -p "$OUT"
for e in ${EXP:-hip_none hip_async hip_legacy hip_all}; do
  echo "[$(date +%T)] $e start" >> "$OUT/steps.txt"
  case $e in
    hipmode_*) m=${e#hipmode_}; timeout -k 10 60 tools/_bin/capture_race_hip "${m%%_*}" "${HIP_SECONDS:-15}" "${m#*_}" \
                 >> "$OUT/results.jsonl" 2>> "$OUT/stderr.txt" ;;  # hipmode_<churn>_<capture mode>
    hip_*) timeout -k 10 60 tools/_bin/capture_race_hip "${e#hip_}" "${HIP_SECONDS:-15}" >> "$OUT/results.jsonl" 2>> "$OUT/stderr.txt" ;;
    libg_*) timeout -k 10 220 python3 tools/capture_race_run.py capture_race 2 CAPTURE_RACE_CHURN="${e#libg_}" \
             TIPS_GRAPHS=1 TIPS_FRESH_WAIT_LIMIT=1000 >> "$OUT/results.jsonl" 2>> "$OUT/stderr.txt" ;;  # replays on
    lib_*) timeout -k 10 220 python3 tools/capture_race_run.py capture_race 2 CAPTURE_RACE_CHURN="${e#lib_}" \
             TIPS_FRESH_WAIT_LIMIT=1000 >> "$OUT/results.jsonl" 2>> "$OUT/stderr.txt" ;;
    opbody_nb_neg) timeout -k 10 220 python3 tools/capture_race_run.py op_body 3 OP_BODY_TENSORS=96 \
                     OP_BODY_NONBLOCKING=1 TIPS_GRAPHS=1 TIPS_GRAPHS_NEGOTIATION=1 >> "$OUT/results.jsonl" 2>> "$OUT/stderr.txt" ;;
    opbody_neg) timeout -k 10 220 python3 tools/capture_race_run.py op_body 3 OP_BODY_TENSORS=96 \
                  TIPS_GRAPHS=1 TIPS_GRAPHS_NEGOTIATION=1 >> "$OUT/results.jsonl" 2>> "$OUT/stderr.txt" ;;
    *) echo "unknown $e" >> "$OUT/steps.txt"; exit 2 ;;
  esac
  rc=$?
  echo "[$(date +%T)] $e rc=$rc" >> "$OUT/steps.txt"
  # (exit 1 = the run finished and counted failures: go on; a crash, stall or time limit ends the call)
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
