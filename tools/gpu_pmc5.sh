#!/bin/bash
# GPU box: PMC passes (tools/pmc_sets.txt, one counter set per run) of one bench workload.
#   tools/gpu_pmc5.sh <tag> <prefix> "<bench args>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
python3 -c "import bench; print(bench.source_sha16())" > $O/source_sha16.txt
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line --output-format csv -d $O/$2/p$i -o run -- \
      python3 bench.py $3 --no-cpu --settle-seconds 0 > $O/$2_p$i.log 2>&1 || exit 1
done < tools/pmc_sets.txt
