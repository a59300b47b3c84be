#!/bin/bash
# GPU box: rocprofv3 PMC passes (one counter set per run) for the headline
# (config 2) and config 4 forward kernels, plus kernel-trace stats for config 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-pmc}
mkdir -p gpurun_out/$TAG
i=0
for cfg in cfg2 cfg4; do
  steps=5; [ $cfg = cfg4 ] && steps=3
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $line --output-format csv -d gpurun_out/$TAG/${cfg}_p$i -o run -- \
        python3 bench.py --config $cfg --steps $steps --warmup 1 --no-cpu > gpurun_out/$TAG/${cfg}_p$i.log 2>&1 || exit 1
  done < "${PMC_FILE:-tools/pmc_sets.txt}"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/cfg4_trace -o run -- \
    python3 bench.py --config cfg4 --steps 10 --warmup 2 --no-cpu > gpurun_out/$TAG/cfg4_trace.log 2>&1
