#!/bin/bash
# r03a: the round's first GPU pass on this tree - parity tests, smoke, bench lines, then the pack
# kernel's launch-size ceiling (tools/pack_ceiling.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r03a PYTEST_TIMEOUT=800 PROFILE=0 bash tools/gpu_round.sh || exit $?
OUT="$PWD/gpurun_out/r03a"
timeout -k 10 240 python -u tools/pack_ceiling.py 7 > "$OUT/pack_ceiling.jsonl" 2> "$OUT/pack_ceiling.err" || exit $?
TIPS_FUSION_THRESHOLD=2147483648 timeout -k 10 240 python -u tools/pack_ceiling.py 7 > "$OUT/pack_ceiling_sizes.jsonl" 2> "$OUT/pack_ceiling_sizes.err"
