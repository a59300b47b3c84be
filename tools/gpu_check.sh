#!/bin/bash
# GPU box: named GPU tests first (TESTS="file::test ..."), then the whole -m gpu suite,
# smoke() and the driver's bench command.  Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-check}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -v -rs --timeout 180 --timeout-method thread > $O/pytest_new.log 2>&1
  rc=$?; echo "pytest rc $rc" >> $O/pytest_new.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
[ "${FULL:-1}" = 1 ] || exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
