#!/bin/bash
# GPU box: A/B of kernel-variant libraries ($VARIANTS, lib<v>.so) on the config-4 forward and config-5 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab4}
mkdir -p $O
for v in $VARIANTS; do
  L=$PWD/densityflows.jl_amd/lib$v.so
  DENSITYFLOWS_HIP_LIB=$L timeout -k 10 200 python bench.py --config cfg4 --steps 20 --warmup 5 --no-cpu --no-exact > $O/cfg4_$v.json 2> $O/cfg4_$v.err || exit 1
  DENSITYFLOWS_HIP_LIB=$L timeout -k 10 200 python bench.py --mode train --config cfg4 --steps 4 --warmup 2 > $O/t5_$v.json 2> $O/t5_$v.err || exit 1
done
for f in $O/*.json; do echo "$f $(python3 -c "import json; print(json.loads(open('$f').read().strip().splitlines()[-1])['value'])")"; done > $O/summary.txt
