#!/bin/bash
# GPU box: one rocprofv3 kernel trace of a bench command under optional env settings.
#   tools/gpu_trace.sh <tag> "<env assignments>" "<bench args>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
env $2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py $3 --no-cpu > $O/prof.json 2> $O/prof.err
