#!/bin/bash
# GPU box: fused-path training tests, then the config-2 train bench and its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-t2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 240 python bench.py --mode train --steps 20 --warmup 5 > $O/train_cfg2.json 2> $O/train_cfg2.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t2 -o run -- \
    python3 bench.py --mode train --steps 10 --warmup 3 > $O/prof_t2.log 2>&1
