#!/bin/bash
# GPU box: parity tests, headline bench, and a rocprofv3 kernel-trace summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 50 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/prof_$TAG.log 2>&1
