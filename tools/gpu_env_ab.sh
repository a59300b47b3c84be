#!/bin/bash
# GPU box: the -m gpu suite on the in-tree build, then an interleaved A/B of one
# environment knob on bench workloads.
#   tools/gpu_env_ab.sh <tag> <VAR> "<value A> <value B>" "<bench args>" ["<bench args>" ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
VAR=$2
VALS=$3
shift 3
mkdir -p $O
if [ "${SKIPTESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
fi
w=0
for args in "$@"; do
  w=$((w+1))
  for rep in 1 2; do
    for v in $VALS; do
      env $VAR=$v timeout -k 10 300 python3 bench.py $args --no-cpu > $O/w${w}_${v}_$rep.json 2> $O/w${w}_${v}_$rep.err || exit 1
    done
  done
done
for f in $O/w*_*.json; do
  python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('%-20s %-40s value %10.3f ms_per_step %.4f' % ('$(basename $f)', d['config']['workload'][:40], d['value'], d['ms_per_step']))
"
done | tee $O/summary.txt
