#!/bin/bash
# PMC passes for the bucket-sum kernel (run on the GPU box). FETCH_SIZE and WRITE_SIZE in
# separate passes (TCC slots), counters only with --kernel-trace-free runs, no sys/runtime traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-pmc}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o bench \
    -- python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 2 ${BENCH_ARGS:-} > "$OUT/pmc_$c.log" 2>&1 || exit $?
done
exit 0
