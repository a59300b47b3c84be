#!/bin/bash
# GPU box: GPU parity tests, then the headline bench under each environment
# setting in $ENVS (space-separated; "-" = none), interleaved twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-envab}
mkdir -p gpurun_out/$TAG
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || exit 1
fi
for rep in 1 2; do
  for e in ${ENVS:--}; do
    if [ "$e" = "-" ]; then envs=""; else envs="$e"; fi
    env $envs timeout -k 10 200 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/$TAG/b_${e//[^A-Za-z0-9_]/_}_$rep.json 2> gpurun_out/$TAG/b_${e//[^A-Za-z0-9_]/_}_$rep.err || exit 1
  done
done
