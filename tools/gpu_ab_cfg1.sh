#!/bin/bash
# GPU box: interleaved A/B of library variants on config 1 (B = 4096 and 2^20).
#   tools/gpu_ab_cfg1.sh <tag> "<libs>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for rep in 1 2; do
  for lib in $2; do
    DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$lib timeout -k 10 240 python3 bench.py --config cfg1 --batch 4096 --steps 500 --warmup 100 --no-cpu \
        > $O/s_${lib%.so}_$rep.json 2> $O/s_${lib%.so}_$rep.err || exit 1
    DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$lib timeout -k 10 240 python3 bench.py --config cfg1 --steps 200 --warmup 50 --no-cpu \
        > $O/l_${lib%.so}_$rep.json 2> $O/l_${lib%.so}_$rep.err || exit 1
  done
done
for f in $O/s_*.json $O/l_*.json; do
  python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('%-36s value %10.3f ms %.5f' % ('$(basename $f)', d['value'], d['ms_per_step']))
"
done | tee $O/summary.txt
