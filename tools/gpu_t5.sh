#!/bin/bash
# GPU box: layer-wise training tests, then the config-5 train bench (+ NOMERGE A/B) and its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-t5}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 180 --timeout-method thread \
    -k "${TESTK:-layerwise or merged or cfg5 or wide or docs or other_act}" > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --mode train --config cfg4 --steps 5 --warmup 2 > $O/train_cfg5.json 2> $O/train_cfg5.err && \
DF_TRAIN_NOMERGE=1 timeout -k 10 300 python bench.py --mode train --config cfg4 --steps 5 --warmup 2 > $O/train_cfg5_nomerge.json 2> $O/train_cfg5_nomerge.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t5 -o run -- \
    python3 bench.py --mode train --config cfg4 --steps 3 --warmup 1 > $O/prof_t5.log 2>&1
