#!/bin/bash
# GPU box: A/B the kernel-variant libraries named in $VARIANTS on the headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-ab}
for v in $VARIANTS; do
  DENSITYFLOWS_HIP_LIB=$PWD/densityflows.jl_amd/lib$v.so timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab_${TAG}_$v.log 2>&1 || exit 1
done
