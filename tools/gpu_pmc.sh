#!/bin/bash
# GPU box: rocprofv3 PMC passes on the headline bench (counters in separate passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-pmc}
mkdir -p gpurun_out/$TAG
if [ ! -f gpurun_out/counters_list.txt ]; then
  timeout -k 10 120 rocprofv3 -L > gpurun_out/$TAG/counters_list.txt 2>&1 || true
fi
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $line --output-format csv -d gpurun_out/$TAG/p$i -o run -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed: $line" >> gpurun_out/$TAG/failed.txt; }
done < "${PMC_FILE:-tools/pmc_sets.txt}"
