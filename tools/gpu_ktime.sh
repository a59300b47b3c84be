#!/bin/bash
# GPU box: per-kernel average time of one workload under several library builds.
#   tools/gpu_ktime.sh <tag> "<bench args>" "<kernel regex>" <lib> [<lib> ...]
# Extra environment for the bench (e.g. DF_TRAIN_NOMERGE=1) is inherited.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; ARGS=$2; PAT=$3
shift 3
mkdir -p $O
for lib in "$@"; do
  DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/${lib%.so} -o run -- python3 bench.py $ARGS --no-cpu --no-exact > $O/${lib%.so}.log 2>&1 || exit 1
  echo "== $lib" >> $O/summary.txt
  grep -E "$PAT" $O/${lib%.so}/run_kernel_stats.csv | cut -d, -f1-4 >> $O/summary.txt
done
cat $O/summary.txt
