#!/bin/bash
# GPU box: rocprofv3 kernel-trace summaries of the config-2 and config-5 train steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-tprof}
mkdir -p gpurun_out/$TAG
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/cfg2 -o run -- \
    python3 bench.py --mode train --steps 10 --warmup 3 > gpurun_out/$TAG/cfg2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/cfg5 -o run -- \
    python3 bench.py --mode train --config cfg4 --steps 3 --warmup 1 > gpurun_out/$TAG/cfg5.log 2>&1
