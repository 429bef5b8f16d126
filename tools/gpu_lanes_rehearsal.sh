#!/bin/bash
# bench.py N=2 over real RCCL ranks sharing the GPU (socket transport): the tuned choice, then
# direct on two transfer lanes against one lane, back to back in one call.
set -e
cd "$(dirname "$0")/.."
export TIPS_VERBOSE=1 TIPS_BENCH_FAKE_HOSTS=1
B="python -u bench.py --gpus 2 --bucket-mib ${MIB:-64} --steps 6 --warmup 1 --no-compare"
timeout -k 10 200 $B > gpurun_out/r02_reh_l3.log 2>&1
TIPS_LANES=2 timeout -k 10 200 $B --algo direct > gpurun_out/r02_reh_l4.log 2>&1
TIPS_LANES=1 timeout -k 10 200 $B --algo direct > gpurun_out/r02_reh_l5.log 2>&1
