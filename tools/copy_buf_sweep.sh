#!/bin/bash
# config 3 at one rank (1 GiB out-of-place allreduce = one contiguous copy): copy_buf_kernel variants
# (TIPS_COPY_BUF_VARIANT 0-4, see kernels.hip launch_copy_buf; the file recorded in profiles/r04/z_copy_buf_sweep.txt ran the old numbering, where 0 = 8 KiB and 1 = 4 KiB tiles) interleaved over 3 rounds, one bench
# process each. gpurun_out/$TAG/copy_buf_sweep.txt
set -e
OUT=gpurun_out/${TAG:-copybuf}
mkdir -p "$OUT"
for round in 1 2 3; do
  for v in ${VARIANTS:-0 1 2 3 4 5 6}; do
    printf 'variant %s ' "$v" >> "$OUT/copy_buf_sweep.txt"
    TIPS_COPY_BUF_VARIANT=$v timeout -k 5 120 python bench.py --workload bucket --no-sub --no-cpu-baseline \
      --steps 20 --warmup 3 2>/dev/null | grep '^{' >> "$OUT/copy_buf_sweep.txt"
  done
done
