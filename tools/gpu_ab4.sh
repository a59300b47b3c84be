#!/bin/bash
# GPU box: gradient + parity tests on the in-tree build, then interleaved A/Bs of the
# in-tree build against densityflows.jl_amd/libdf_old.so.
#   tools/gpu_ab4.sh <tag>    (env: TESTS, AB = "cfg5 cfg1 cfg2 train2 cfg4", REPS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ -n "${TESTS-tests/test_gpu_train.py tests/test_gpu_parity.py}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS-tests/test_gpu_train.py tests/test_gpu_parity.py} -m gpu -x -q \
      --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
run() {  # <name> <lib> <rep> <bench args>   (lib "env": the in-tree build under $ABENV)
  local so=$2 tag=${2%.so} envs=""
  if [ "$2" = env ]; then so=libdensityflows_hip.so; envs="$ABENV"; fi
  if [ "$2" = env2 ]; then so=libdensityflows_hip.so; envs="$ABENV2"; fi
  env $envs DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$so timeout -k 10 300 python3 bench.py $4 --no-cpu \
      > $O/$1_${tag}_$3.json 2> $O/$1_${tag}_$3.err
}
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS:-libdf_old.so libdensityflows_hip.so} ${ABENV:+env} ${ABENV2:+env2}; do
    for w in ${AB:-cfg5 cfg1}; do
      case $w in
        cfg5) run cfg5 $lib $rep "--mode train --config cfg4 --steps 5 --warmup 2" || exit 1 ;;
        cfg1) run cfg1 $lib $rep "--config cfg1 --steps 300 --warmup 50" || exit 1 ;;
        cfg1s) run cfg1s $lib $rep "--config cfg1 --batch 4096 --steps 300 --warmup 50" || exit 1 ;;
        cfg2) run cfg2 $lib $rep "--steps 200 --warmup 50 --no-exact" || exit 1 ;;
        train2) run train2 $lib $rep "--mode train --steps 20 --warmup 5" || exit 1 ;;
        cfg4) run cfg4 $lib $rep "--config cfg4 --steps 10 --warmup 3 --no-exact" || exit 1 ;;
      esac
    done
  done
done
if [ -n "${PROF:-}" ]; then  # kernel trace of the in-tree build on config 1 at B = 4096
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o cfg1s -- \
      python3 $GRAFT_REPO_ROOT/bench.py --config cfg1 --batch 4096 --steps 300 --warmup 50 --no-cpu --no-clock \
      > $GRAFT_REPO_ROOT/$O/prof_cfg1s.json 2> $GRAFT_REPO_ROOT/$O/prof_cfg1s.err || exit 1
  cd $GRAFT_REPO_ROOT
  python3 tools/kgap.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/kgap_cfg1s.txt || exit 1
  cat $O/kgap_cfg1s.txt
fi
for f in $O/*_lib*.json $O/*_env_*.json $O/*_env2_*.json; do
  [ -f "$f" ] || continue
  python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]);c=d.get('clock') or {}
print('%-44s value %9.3f ms_per_step %.4f kernel_ms %s mcyc %s ghz %s' % ('$(basename $f)', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'), c.get('kernel_mcycles_per_launch'), c.get('ghz_median')))
"
done | tee $O/summary.txt
