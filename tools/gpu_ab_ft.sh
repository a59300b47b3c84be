#!/bin/bash
# GPU box: interleaved A/B of library variants on the config-2 forward (headline workload,
# 200 / 50 steps) and the config-2 train step.
#   tools/gpu_ab_ft.sh <tag> "<libs>"   (libs: .so files under densityflows.jl_amd/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for rep in 1 2; do
  for lib in $2; do
    DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$lib timeout -k 10 240 python3 bench.py --steps 200 --warmup 50 --no-cpu \
        > $O/fwd_${lib%.so}_$rep.json 2> $O/fwd_${lib%.so}_$rep.err || exit 1
    DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$lib timeout -k 10 240 python3 bench.py --mode train --steps 20 --warmup 5 --no-cpu \
        > $O/trn_${lib%.so}_$rep.json 2> $O/trn_${lib%.so}_$rep.err || exit 1
  done
done
for f in $O/fwd_*.json $O/trn_*.json; do
  python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
c=d.get('clock',{})
print('%-36s value %9.3f ms %.4f Mcyc %s GHz %s' % ('$(basename $f)', d['value'], d['ms_per_step'], c.get('kernel_mcycles_per_launch'), c.get('ghz_median')))
"
done | tee $O/summary.txt
