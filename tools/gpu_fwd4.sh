#!/bin/bash
# GPU box: forward parity tests, then the config-4 (and headline) forward benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-f4}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 240 python bench.py --config cfg4 --steps 20 --warmup 10 --no-cpu > $O/cfg4.json 2> $O/cfg4.err && \
timeout -k 10 240 python bench.py --config cfg4 --steps 20 --warmup 10 --no-cpu > $O/cfg4b.json 2> $O/cfg4b.err && \
timeout -k 10 240 python bench.py --no-cpu > $O/cfg2.json 2> $O/cfg2.err
