#!/bin/bash
# GPU box: the whole -m gpu suite (no -x), then a headline bench and its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-t2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -s --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python bench.py --cpu-seconds 5 > $O/bench.json 2> $O/bench.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --no-cpu > $O/prof.log 2>&1
