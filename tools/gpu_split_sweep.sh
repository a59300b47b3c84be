#!/bin/bash
# GPU box: headline SPLIT kernel under LDS budgets / resident tiles (env knobs, no rebuild).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-sw}
mkdir -p $O
for kb in ${KBS:-80 96 112 128 160}; do
  for t in ${TS:-0 2 4 6 8}; do
    if [ $t = 0 ]; then unset DF_TILES; else export DF_TILES=$t; fi
    DF_SPLIT_LDS_KB=$kb DF_DEBUG_LAUNCH=1 timeout -k 10 60 python bench.py --steps 100 --warmup 20 --no-cpu --no-exact \
        > $O/kb${kb}_t${t}.json 2> $O/kb${kb}_t${t}.err || exit 1
  done
done
unset DF_TILES
for f in $O/kb*.json; do echo "$f $(python3 -c "import json,sys; print(json.loads(open('$f').read().strip().splitlines()[-1])['value'])") $(grep -m1 '\[df\]' ${f%.json}.err | sed 's/.*tiles/tiles/')"; done > $O/summary.txt
