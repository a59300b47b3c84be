#!/bin/bash
# GPU box: config 1 at small batches on library variants built with fewer waves per
# workgroup (tools/build_variant.sh wN "-DDF_BLOCK_WAVES=N").
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-cfgw}; mkdir -p $O
for lib in libdensityflows_hip w1 w2 w4; do
  so=densityflows.jl_amd/$lib.so; [ $lib != libdensityflows_hip ] && so=densityflows.jl_amd/libdf_$lib.so
  for b in 4096 65536; do
    for t in 2 4; do
      DENSITYFLOWS_HIP_LIB=$so DF_TILES=$t timeout -k 10 120 python3 bench.py --config cfg1 --batch $b --steps 300 --warmup 50 --no-cpu > $O/${lib}_b${b}_t$t.json 2>$O/${lib}_b${b}_t$t.err || exit 1
    done
  done
done
for f in $O/*.json; do python3 -c "
import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);c=d.get('clock') or {}
print('$f', d['config'].get('per_gpu_batch'), round(d['value'],1), d['roofline'].get('kernel_ms'), c.get('kernel_mcycles_per_launch'), c.get('workgroup_slots'))"; done | tee $O/summary.txt
