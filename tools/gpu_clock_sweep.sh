#!/bin/bash
# GPU box: headline throughput vs warm-up / timed-step counts (DVFS settling).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/clk
for sw in "20 3" "50 5" "200 50" "500 200" "1000 500"; do
  set -- $sw
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu > gpurun_out/clk/s$1_w$2.json 2>/dev/null || exit 1
done
