#!/bin/bash
# GPU box: interleaved A/B of library variants on the config-4 forward (wide SPLIT kernel)
# and the config-5 train step.
#   tools/gpu_ab_cfg4.sh <tag> "<libs>"   (libs: .so files under densityflows.jl_amd/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for rep in 1 2; do
  for lib in $2; do
    DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$lib timeout -k 10 240 python3 bench.py --config cfg4 --steps 20 --warmup 10 --no-cpu \
        > $O/c4_${lib%.so}_$rep.json 2> $O/c4_${lib%.so}_$rep.err || exit 1
    DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$lib timeout -k 10 300 python3 bench.py --mode train --config cfg4 --steps 5 --warmup 2 --no-cpu \
        > $O/c5_${lib%.so}_$rep.json 2> $O/c5_${lib%.so}_$rep.err || exit 1
  done
done
for f in $O/c4_*.json $O/c5_*.json; do
  python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('%-36s value %9.3f ms %.4f' % ('$(basename $f)', d['value'], d['ms_per_step']))
"
done | tee $O/summary.txt
