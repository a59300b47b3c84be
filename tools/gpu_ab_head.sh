#!/bin/bash
# GPU box: A/B of kernel-variant libraries ($VARIANTS, lib<v>.so) on the headline forward.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-abh}
mkdir -p $O
for v in $VARIANTS; do
  DENSITYFLOWS_HIP_LIB=$PWD/densityflows.jl_amd/lib$v.so timeout -k 10 200 python bench.py --no-cpu --no-exact > $O/h_$v.json 2> $O/h_$v.err || exit 1
done
for f in $O/*.json; do echo "$f $(python3 -c "import json; print(json.loads(open('$f').read().strip().splitlines()[-1])['value'])")"; done > $O/summary.txt
