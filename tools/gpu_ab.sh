#!/bin/bash
# GPU box: interleaved A/B of library builds on one workload.
#   tools/gpu_ab.sh <tag> "<bench args>" <lib> [<lib> ...]
# <lib> is a .so under densityflows.jl_amd/ (libdensityflows_hip.so = the in-tree build).
# Optional: TESTLIB=<lib> runs the -m gpu suite against that build first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
ARGS=$2
shift 2
mkdir -p $O
if [ -n "${TESTLIB:-}" ]; then
  DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$TESTLIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
      --timeout 180 --timeout-method thread > $O/pytest_$TESTLIB.log 2>&1 || exit 1
fi
for rep in 1 2; do
  for lib in "$@"; do
    DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$lib timeout -k 10 300 python3 bench.py $ARGS --no-cpu --no-exact \
        > $O/${lib%.so}_$rep.json 2> $O/${lib%.so}_$rep.err || exit 1
  done
done
for lib in "$@"; do
  for rep in 1 2; do
    python3 -c "
import json,sys
d=json.loads(open('$O/${lib%.so}_$rep.json').read().strip().splitlines()[-1])
c=d.get('clock') or {}
print('%-28s rep $rep value %9.3f kernel_ms %.4f ghz %s Mcyc %s' % ('$lib', d['value'], d['roofline']['kernel_ms'], c.get('ghz_median'), c.get('kernel_mcycles_per_launch')))
"
  done
done | tee $O/summary.txt
