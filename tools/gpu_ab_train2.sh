#!/bin/bash
# GPU box: A/B of kernel-variant libraries ($VARIANTS, lib<v>.so) on the config-2 train step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-abt2}
mkdir -p $O
for v in $VARIANTS; do
  DENSITYFLOWS_HIP_LIB=$PWD/densityflows.jl_amd/lib$v.so timeout -k 10 200 python bench.py --mode train --steps 20 --warmup 5 > $O/t2_$v.json 2> $O/t2_$v.err || exit 1
done
for f in $O/*.json; do echo "$f $(python3 -c "import json; print(json.loads(open('$f').read().strip().splitlines()[-1])['value'])")"; done > $O/summary.txt
