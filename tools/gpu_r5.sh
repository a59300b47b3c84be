#!/bin/bash
# GPU box, round 5: named GPU tests (TESTS=...), then interleaved config-5 train-step A/B of
# the H0-free sweep (default) against the kept-H0 sweep (DF_TRAIN_H0=1), then a kernel
# trace of the default.  Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -v -rs --timeout 180 --timeout-method thread > $O/pytest_new.log 2>&1
  rc=$?; echo "pytest rc $rc" >> $O/pytest_new.log
  [ $rc -ne 0 ] && exit $rc
fi
[ "${AB:-1}" = 1 ] || exit 0
for r in 1 2; do
  for h in 0 1; do
    DF_TRAIN_H0=$h timeout -k 10 300 python bench.py --mode train --config cfg4 --steps 5 --warmup 2 --no-cpu \
      > $O/t5_h0${h}_$r.json 2> $O/t5_h0${h}_$r.err || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t5 -o run -- \
    python3 bench.py --mode train --config cfg4 --steps 3 --warmup 1 --no-cpu > $O/prof_t5.log 2>&1
