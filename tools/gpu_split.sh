#!/bin/bash
# GPU box: SPLIT (bf16x3) variant check — parity subset, then headline A/B against the exact-f32 FAST kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/split
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "golden or strict or fast_variant or ragged or inplace or sample or theta or folded" > $O/pytest.log 2>&1
echo "pytest rc $?" >> $O/pytest.log
DF_DEBUG_LAUNCH=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $O/dbg.json 2> $O/dbg.err
timeout -k 10 120 python bench.py --no-cpu > $O/bench_split.json 2> $O/bench_split.err && \
DF_F32_EXACT=1 timeout -k 10 120 python bench.py --no-cpu > $O/bench_exact.json 2> $O/bench_exact.err
