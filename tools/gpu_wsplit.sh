#!/bin/bash
# GPU box: wide SPLIT kernel — parity subset, training tests on the wide/cfg5 nets, cfg4 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-ws}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 120 --timeout-method thread \
    -k "golden or strict or split or wide or full_size or deterministic or inplace" > $O/pytest.log 2>&1
echo "pytest rc $?" >> $O/pytest.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -v -s --timeout 120 --timeout-method thread \
    -k "wide or cfg5" > $O/pytest_train.log 2>&1
echo "pytest rc $?" >> $O/pytest_train.log
DF_DEBUG_LAUNCH=1 timeout -k 10 120 python bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu --no-exact > $O/dbg.json 2> $O/dbg.err
timeout -k 10 240 python bench.py --config cfg4 --steps 20 --warmup 5 --no-cpu > $O/cfg4.json 2> $O/cfg4.err && \
timeout -k 10 300 python bench.py --mode train --config cfg4 --steps 5 --warmup 2 > $O/train_cfg5.json 2> $O/train_cfg5.err
