#!/bin/bash
# GPU box: full GPU test suite against the first library variant in $VARIANTS, then
# the headline bench A/B (alternating, twice) for every variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abf
export TMPDIR=/tmp
first=${VARIANTS%% *}
DENSITYFLOWS_HIP_LIB=$PWD/densityflows.jl_amd/lib$first.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abf/pytest_$first.log 2>&1 || exit 1
for rep in 1 2; do
for v in $VARIANTS; do
  DENSITYFLOWS_HIP_LIB=$PWD/densityflows.jl_amd/lib$v.so timeout -k 10 200 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/abf/bench_${v}_$rep.json 2> gpurun_out/abf/bench_${v}_$rep.err || exit 1
done
done
