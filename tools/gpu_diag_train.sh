#!/bin/bash
# GPU box: training diagnostics — config-5 step with unmerged sweep launches (per-kernel times),
# and PMC of the config-2 fused training kernel (one counter set per run).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-dt}
mkdir -p $O
DF_TRAIN_NOMERGE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t5_nomerge -o run -- \
    python3 bench.py --mode train --config cfg4 --steps 3 --warmup 1 > $O/prof_t5_nomerge.log 2>&1 || exit 1
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line --output-format csv -d $O/pmc_t2/p$i -o run -- \
      python3 bench.py --mode train --steps 3 --warmup 1 > $O/pmc_t2_p$i.log 2>&1 || exit 1
done < tools/pmc_sets.txt
