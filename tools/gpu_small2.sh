#!/bin/bash
# GPU box: the small-batch kernel — GPU suite, then config 1 across batch sizes with the
# small kernel on / off (DF_SMALL_MAX=0), and the headline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-small2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest ${PYTESTS:-tests} -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc $rc" >> $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for b in ${BATCHES:-256 4096 16384 32768 65536}; do
  for sm in on off; do
    env_=""; [ $sm = off ] && env_="DF_SMALL_MAX=0"
    env $env_ timeout -k 10 120 python3 bench.py --config cfg1 --batch $b --steps 300 --warmup 50 --no-cpu > $O/cfg1_b${b}_$sm.json 2>$O/cfg1_b${b}_$sm.err || exit 1
  done
done
timeout -k 10 120 python3 bench.py --config cfg1 --batch 4096 --steps 300 --warmup 50 --cpu-seconds 10 > $O/cfg1_4096_cpu.json 2>$O/cfg1_4096_cpu.err || exit 1
timeout -k 10 120 python3 bench.py --steps 100 --warmup 20 --no-cpu --no-exact > $O/cfg2.json 2>$O/cfg2.err || exit 1
for f in $O/*.json; do python3 -c "
import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);c=d.get('clock') or {}
print('$f', d['config'].get('per_gpu_batch'), round(d['value'],1), d['roofline'].get('kernel_ms'), c.get('kernel_mcycles_per_launch'), (d.get('cpu_baseline') or {}).get('value'))"; done | tee $O/summary.txt
# interleaved A/B against the previous build (densityflows.jl_amd/libdf_old.so), if present
if [ -f densityflows.jl_amd/libdf_old.so ]; then
  for r in 1 2 3; do
    for lib in old new; do
      so=densityflows.jl_amd/libdensityflows_hip.so; [ $lib = old ] && so=densityflows.jl_amd/libdf_old.so
      DENSITYFLOWS_HIP_LIB=$so timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --no-cpu --no-exact > $O/ab_cfg2_${lib}_$r.json 2>/dev/null || exit 1
      DENSITYFLOWS_HIP_LIB=$so timeout -k 10 120 python3 bench.py --config cfg1 --steps 200 --warmup 50 --no-cpu > $O/ab_cfg1_${lib}_$r.json 2>/dev/null || exit 1
    done
  done
  for f in $O/ab_*.json; do python3 -c "
import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);c=d.get('clock') or {}
print('$f', round(d['value'],1), d['roofline'].get('kernel_ms'), c.get('kernel_mcycles_per_launch'), c.get('ghz_median'))"; done | tee $O/ab_summary.txt
fi
