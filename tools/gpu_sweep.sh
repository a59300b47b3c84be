#!/bin/bash
# GPU box: headline launch-shape sweep of the in-tree build — tiles per wave (DF_TILES)
# and SPLIT stage size (DF_SPLIT_LDS_KB), interleaved, plus the launch shape the
# library picks by itself (DF_DEBUG_LAUNCH=1).
#   tools/gpu_sweep.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-sweep}
mkdir -p $O
DF_DEBUG_LAUNCH=1 timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-exact --no-clock \
    > $O/debug.json 2> $O/debug.err || exit 1
grep "\[df\]" $O/debug.err | sort | uniq -c | head -5
for rep in 1 2; do
  for v in "" "DF_TILES=2" "DF_TILES=4" "DF_TILES=6" "DF_TILES=8" "DF_SPLIT_LDS_KB=48" "DF_SPLIT_LDS_KB=96"; do
    tag=${v:-default}
    env $v timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --no-cpu --no-exact \
        > $O/${tag}_$rep.json 2> $O/${tag}_$rep.err || exit 1
  done
done
for f in $O/*_[12].json; do
  python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]);c=d.get('clock') or {}
print('%-40s value %9.2f kernel_ms %s mcyc %s ghz %s' % ('$(basename $f)', d['value'], d['roofline'].get('kernel_ms'), c.get('kernel_mcycles_per_launch'), c.get('ghz_median')))
"
done | tee $O/summary.txt
