#!/bin/bash
# GPU box: the training-kernel A/Bs of one round (after tools/gpu_round3.sh when PASS is set).
#   tools/gpu_ab_train.sh <tag> "<cfg2 libs>" "<cfg5 libs>" [<lib whose gradient tests run first>]
# Libraries are .so files under densityflows.jl_amd/ (libdensityflows_hip.so = the in-tree build).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ -n "${PASS:-}" ]; then
  NOPMC=1 bash tools/gpu_round3.sh $PASS || exit 1
fi
if [ -n "${4:-}" ]; then
  DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$4 timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q \
      --timeout 180 --timeout-method thread > $O/pytest_$4.log 2>&1
  rc=$?
  # a failing candidate leaves the A/B (a fault or time-out ends the call)
  if [ $rc -eq 1 ]; then set -- "$1" "$2" "${3//$4/}"; elif [ $rc -ne 0 ]; then exit $rc; fi
fi
run() {  # <cfg> <lib> <rep> <bench args>
  DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$2 timeout -k 10 300 python3 bench.py $4 --no-cpu \
      > $O/$1_${2%.so}_$3.json 2> $O/$1_${2%.so}_$3.err
}
for rep in 1 2; do
  for lib in $2; do run cfg2 $lib $rep "--mode train --steps 20 --warmup 5" || exit 1; done
  for lib in $3; do run cfg5 $lib $rep "--mode train --config cfg4 --steps 5 --warmup 2" || exit 1; done
done
for f in $O/cfg*_*.json; do
  python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('%-48s value %9.3f ms_per_step %.3f' % ('$(basename $f)', d['value'], d['ms_per_step']))
"
done | tee $O/summary.txt
