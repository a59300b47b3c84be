#!/bin/bash
# GPU box: LDS-conflict counters of the config-5 training kernels for library variants.
#   tools/gpu_ldsc.sh <tag> <lib>...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for lib in "$@"; do
  DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$lib timeout -s KILL 120 rocprofv3 --kernel-trace \
      --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv \
      -d $O/${lib%.so}/p1 -o run -- python3 bench.py --mode train --config cfg4 --steps 1 --warmup 1 --no-cpu \
      --settle-seconds 0 > $O/${lib%.so}.log 2>&1 || exit 1
done
