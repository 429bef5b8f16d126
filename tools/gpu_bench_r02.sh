set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r02_bench_n1.jsonl 2> gpurun_out/r02_bench_n1.err || exit 1
timeout -k 10 200 python -u bench.py --workload fused1000 > gpurun_out/r02_bench_n1_fused1000.jsonl 2> gpurun_out/r02_f.err || exit 2
timeout -k 10 200 python -u bench.py --workload resnet50 > gpurun_out/r02_bench_n1_resnet50.jsonl 2> gpurun_out/r02_r.err || exit 3
TIPS_BENCH_FAKE_HOSTS=1 timeout -k 10 300 python -u bench.py --gpus 2 --bucket-mib 64 --steps 5 --warmup 2 > gpurun_out/r02_rehearsal_n2.jsonl 2> gpurun_out/r02_n2.err || exit 4
echo done
