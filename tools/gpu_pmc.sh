#!/bin/bash
# GPU box: rocprofv3 PMC passes (tools/pmc_sets.txt, one counter set per run) of one bench
# workload, plus a kernel trace of it.
#   tools/gpu_pmc.sh <tag> "<bench args>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; ARGS=$2
mkdir -p $O
python3 -c "import bench; print(bench.source_sha16())" > $O/source_sha16.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py $ARGS --no-cpu --no-exact > $O/trace.log 2>&1 || exit 1
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line --output-format csv -d $O/p$i -o run -- \
      python3 bench.py $ARGS --no-cpu --no-exact > $O/p$i.log 2>&1 || { echo "pass $i failed: $line"; tail -3 $O/p$i.log; }
done < tools/pmc_sets.txt
exit 0
