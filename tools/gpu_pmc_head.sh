#!/bin/bash
# GPU box: headline bench (SPLIT kernel + exact-f32 side timing), split parity subset,
# kernel trace, and PMC passes (one counter set per run) of the headline kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-ph}
mkdir -p $O
python3 -c "import bench; print(bench.source_sha16())" > $O/source_sha16.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread \
    -k "golden or strict or split or fast_variant" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --cpu-seconds 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --no-cpu --no-exact > $O/prof.log 2>&1 || exit 1
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $line --output-format csv -d $O/pmc/p$i -o run -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu --no-exact > $O/pmc_p$i.log 2>&1 || exit 1
done < tools/pmc_sets.txt
