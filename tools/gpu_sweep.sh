#!/bin/bash
# GPU box: headline bench over a list of environment settings ($ENVS, "-" = none),
# one JSON per setting under gpurun_out/$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-sweep}
mkdir -p gpurun_out/$TAG
for e in ${ENVS:--}; do
  if [ "$e" = "-" ]; then envs=""; else envs="${e//,/ }"; fi
  env $envs timeout -k 10 120 python bench.py --no-cpu --steps ${STEPS:-200} --warmup ${WARM:-50} ${BENCH_ARGS:-} > gpurun_out/$TAG/b_${e//[^A-Za-z0-9_]/_}.json 2> gpurun_out/$TAG/b_${e//[^A-Za-z0-9_]/_}.err || exit 1
done
