#!/bin/bash
# One round's profiles on the GPU box, each GPU step under its own time limit, stopping at the first
# failure. rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs: one TCC group each, no
# traces beside the counters) for the dominant kernel of every bench line:
#   config 2      sum2_buf_kernel     bench.py (the N = 1 headline)
#   config 3, N=1 copy_buf_kernel     bench.py --workload bucket --no-sub
#   configs 4, 5  copy_segs_kernel    tools/pack_ceiling.py --only=configN/pack (the per-bucket pack launches)
# then the kernel trace of the headline (--kernel-trace --stats) for the dispatch-time cross-check.
# Output: gpurun_out/$TAG/; summarise with tools/pmc_traffic.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-pmcround}"
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # name counter cmd...
  local name=$1 c=$2
  shift 2
  echo "[$(date +%T)] $name $c" >> "$OUT/steps.txt"
  timeout -s KILL 240 rocprofv3 --pmc "$c" --output-format csv -d "$OUT/${name}_$c" -o run -- "$@" \
    > "$OUT/${name}_$c.log" 2>&1 || { echo "[$(date +%T)] $name $c rc=$?" >> "$OUT/steps.txt"; exit 1; }
}
for c in FETCH_SIZE WRITE_SIZE; do
  pass config2 $c python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 2
  pass bucket $c python3 bench.py --workload bucket --no-sub --no-cpu-baseline --steps 10 --warmup 2
  pass config4 $c python3 tools/pack_ceiling.py 3 --only=config4/pack
  pass config5 $c python3 tools/pack_ceiling.py 3 --only=config5/pack
done
echo "[$(date +%T)] kernel trace" >> "$OUT/steps.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py \
  --no-sub --no-cpu-baseline --no-extras --steps 200 --warmup 20 > "$OUT/trace.log" 2>&1 || exit 1
echo "[$(date +%T)] done" >> "$OUT/steps.txt"
