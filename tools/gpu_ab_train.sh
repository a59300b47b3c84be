#!/bin/bash
# GPU box: A/B the library variants named in $VARIANTS on the config-5 train step
# (and the GPU training tests against the first variant).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
first=${VARIANTS%% *}
DENSITYFLOWS_HIP_LIB=$PWD/densityflows.jl_amd/lib$first.so timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_train_$first.log 2>&1 || exit 1
for rep in 1 2; do
for v in $VARIANTS; do
  DENSITYFLOWS_HIP_LIB=$PWD/densityflows.jl_amd/lib$v.so timeout -k 10 200 python bench.py --mode train --config cfg4 --steps 6 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/ab/train5_${v}_$rep.json 2> gpurun_out/ab/train5_${v}_$rep.err || exit 1
done
done
for v in $VARIANTS; do
  DENSITYFLOWS_HIP_LIB=$PWD/densityflows.jl_amd/lib$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof_$v -o run -- python3 bench.py --mode train --config cfg4 --steps 2 --warmup 1 > gpurun_out/ab/prof_$v.log 2>&1 || exit 1
done
