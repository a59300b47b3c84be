#!/bin/bash
# GPU box: training tests (layer-wise / wide nets) and the config-5 step with its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-lt}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -v -s --timeout 150 --timeout-method thread > $O/pytest_train.log 2>&1
echo "pytest rc $?" >> $O/pytest_train.log
timeout -k 10 300 python bench.py --mode train --config cfg4 --steps 5 --warmup 2 > $O/train_cfg5.json 2> $O/train_cfg5.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t5 -o run -- \
    python3 bench.py --mode train --config cfg4 --steps 3 --warmup 1 > $O/prof_t5.log 2>&1
