#!/bin/bash
# The driver's N > 1 command (torch.distributed.run, one rank per process) rehearsed on the box's one
# GPU: N RCCL ranks over the socket transport (TIPS_BENCH_FAKE_HOSTS=1), heartbeat file while the
# comparisons run. N=${N:-4}. Output: gpurun_out/$TAG/rehearsal_n$N.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${N:-4}
OUT="$PWD/gpurun_out/${TAG:-rehearsal}"
mkdir -p "$OUT"
( while sleep 45; do date +%T >> "$OUT/heartbeat.txt"; done ) &
HB=$!
TIPS_BENCH_FAKE_HOSTS=1 timeout -k 10 ${REHEARSAL_TIMEOUT:-560} python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus $N --steps 3 --warmup 1 \
  > "$OUT/rehearsal_n$N.log" 2>&1
rc=$?
kill $HB
exit $rc
