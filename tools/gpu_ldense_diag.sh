#!/bin/bash
# GPU box: config-5 step kernel traces of the in-tree build and of a diagnostic build
# (densityflows.jl_amd/libdf_noxbar.so: the W1ᵀδ1 epilogue without x̄ = W0ᵀδ0, wrong
# gradients) — the x̄ share of the W1ᵀδ1 kernel's time.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-ldiag}
mkdir -p $O
for lib in libdensityflows_hip.so libdf_noxbar.so; do
  cd /tmp && DENSITYFLOWS_HIP_LIB=$GRAFT_REPO_ROOT/densityflows.jl_amd/$lib timeout -k 10 300 rocprofv3 --kernel-trace \
      --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/${lib%.so} -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --mode train --config cfg4 --steps 3 --warmup 1 --no-cpu \
      > $GRAFT_REPO_ROOT/$O/${lib%.so}.json 2> $GRAFT_REPO_ROOT/$O/${lib%.so}.err || exit 1
  cd $GRAFT_REPO_ROOT
  f=$(find $O/${lib%.so} -name "run_kernel_stats.csv" | head -1)
  echo "== $lib"; head -8 $f | cut -d, -f1-4
done
