#!/bin/bash
# GPU box: config-1 small-batch work — phase stamps (libdf_ph.so), parity subset, cfg1 benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-small}; mkdir -p $O
DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/libdf_ph.so timeout -k 10 120 python3 tools/phase_stamps.py cfg1 4096 > $O/phase_cfg1.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_julia_replay.py -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc $rc" >> $O/pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for b in 4096 1048576; do
  timeout -k 10 120 python3 bench.py --config cfg1 --batch $b --steps 300 --warmup 50 --no-cpu > $O/cfg1_b$b.json 2>$O/cfg1_b$b.err || exit 1
done
timeout -k 10 120 python3 bench.py --steps 100 --warmup 20 --no-cpu --no-exact > $O/cfg2.json 2>$O/cfg2.err || exit 1
for f in $O/*.json; do python3 -c "
import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);c=d.get('clock') or {}
print('$f', d['config'].get('per_gpu_batch'), round(d['value'],1), d['roofline'].get('kernel_ms'), c.get('kernel_mcycles_per_launch'))"; done | tee $O/summary.txt
