#!/bin/bash
# GPU box: A/B of kernel-variant libraries ($VARIANTS, densityflows.jl_amd/lib<v>.so) on the
# headline forward, config-4 forward and both training steps, interleaved A B A B.
# Optional: $PROBE (a tools/probe binary run first), $TESTS=1 (the -m gpu suite on the in-tree lib).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-aball}
mkdir -p $O
if [ -n "$PROBE" ]; then timeout -k 10 60 ./tools/probe/$PROBE > $O/probe.log 2>&1 || exit 1; fi
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
fi
for rep in 1 2; do
  for v in $VARIANTS; do
    L=$PWD/densityflows.jl_amd/lib$v.so
    DENSITYFLOWS_HIP_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-exact > $O/h_${v}_$rep.json 2> $O/h_${v}_$rep.err || exit 1
    DENSITYFLOWS_HIP_LIB=$L timeout -k 10 200 python bench.py --config cfg4 --steps 20 --warmup 5 --no-cpu --no-exact > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || exit 1
    DENSITYFLOWS_HIP_LIB=$L timeout -k 10 200 python bench.py --mode train --steps 20 --warmup 5 --no-cpu > $O/t2_${v}_$rep.json 2> $O/t2_${v}_$rep.err || exit 1
    DENSITYFLOWS_HIP_LIB=$L timeout -k 10 200 python bench.py --mode train --config cfg4 --steps 5 --warmup 2 --no-cpu > $O/t5_${v}_$rep.json 2> $O/t5_${v}_$rep.err || exit 1
  done
done
for f in $O/*.json; do echo "$f $(python3 -c "import json; print(json.loads(open('$f').read().strip().splitlines()[-1])['value'])")"; done > $O/summary.txt
