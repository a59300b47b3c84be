#!/bin/bash
# GPU box: the round-end checks the driver runs — the -m gpu suite, smoke(), and the
# driver's bench command — on the current in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rs --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log && \
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err && \
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['clock'], d['clock_settle'], d.get('f32_exact_kernel'))"
