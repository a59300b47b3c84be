#!/bin/bash
# GPU box: training tests, then the config-2 train step (fused per-net kernels) with its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-ft}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -v -s --timeout 150 --timeout-method thread > $O/pytest_train.log 2>&1
echo "pytest rc $?" >> $O/pytest_train.log
timeout -k 10 240 python bench.py --mode train --steps 20 --warmup 5 > $O/train_cfg2.json 2> $O/train_cfg2.err && \
DF_F32_EXACT=1 timeout -k 10 240 python bench.py --mode train --steps 20 --warmup 5 > $O/train_cfg2_exact.json 2> $O/train_cfg2_exact.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t2 -o run -- \
    python3 bench.py --mode train --steps 10 --warmup 3 > $O/prof_t2.log 2>&1
