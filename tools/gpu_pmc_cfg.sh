#!/bin/bash
# GPU box: rocprofv3 PMC passes (one counter set per run, $PMC_FILE) on one bench config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-pmc}
mkdir -p gpurun_out/$TAG
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $line --output-format csv -d gpurun_out/$TAG/p$i -o run -- \
      python3 bench.py --steps ${STEPS:-20} --warmup ${WARM:-20} --no-cpu ${BENCH_ARGS:-} > gpurun_out/$TAG/p$i.log 2>&1 || exit 1
done < "${PMC_FILE:-tools/pmc_quick2.txt}"
