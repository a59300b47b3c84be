#!/bin/bash
# GPU box: kernel-trace stats of the config-5 train step for each library variant in $VARIANTS
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pv
export TMPDIR=/tmp
for v in $VARIANTS; do
  DENSITYFLOWS_HIP_LIB=$PWD/densityflows.jl_amd/lib$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pv/prof_$v -o run -- python3 bench.py --mode train --config cfg4 --steps 2 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/pv/prof_$v.log 2>&1 || exit 1
done
