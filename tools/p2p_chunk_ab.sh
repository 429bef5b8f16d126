#!/bin/bash
# bench.py at N = 2 over the socket transport (TIPS_BENCH_FAKE_HOSTS=1), the default RCCL p2p
# chunk vs larger ones: does NCCL_P2P_NET_CHUNKSIZE explain the gap between ncclAllReduce and the
# library's send/recv schedules on this transport (compare_algbw_gib_s)? Output: gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-p2pchunk}"
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for c in ${CHUNKS:-default 524288 2097152}; do
  i=$((i + 1))
  if [ "$c" = default ]; then unset NCCL_P2P_NET_CHUNKSIZE; else export NCCL_P2P_NET_CHUNKSIZE=$c; fi
  TIPS_BENCH_FAKE_HOSTS=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-sub \
    --no-cpu-baseline > "$OUT/n2_${i}_$c.log" 2>&1 || exit 1
done
