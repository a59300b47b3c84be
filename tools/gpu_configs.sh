#!/bin/bash
# GPU box: secondary configs and modes of bench.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-cfg}
timeout -k 10 200 python bench.py --config cfg1 --batch 4096 --steps 200 --warmup 10 --cpu-seconds 5 > gpurun_out/bench_${TAG}_cfg1_4096.log 2>&1 && \
timeout -k 10 200 python bench.py --config cfg1 --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_${TAG}_cfg1_1M.log 2>&1 && \
timeout -k 10 300 python bench.py --config cfg4 --batch 262144 --steps 10 --warmup 2 --cpu-seconds 10 > gpurun_out/bench_${TAG}_cfg4.log 2>&1 && \
timeout -k 10 200 python bench.py --mode nll --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_${TAG}_nll.log 2>&1 && \
DF_FORCE_GENERIC=1 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_${TAG}_cfg2_generic.log 2>&1
