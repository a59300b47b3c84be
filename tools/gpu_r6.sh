#!/bin/bash
# GPU box, round 6: bitwise output comparison of two builds (tools/dump_outputs.py; env
# OLD, default libdf_old.so, and NEW, default the in-tree libdensityflows_hip.so), then
# tools/gpu_ab4.sh (tests + interleaved A/B benches).
#   tools/gpu_r6.sh <tag>   (env as gpu_ab4.sh; NODUMP=1 skips the comparison)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ "${NODUMP:-0}" != 1 ]; then
  DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/${OLD:-libdf_old.so} timeout -k 10 240 python3 tools/dump_outputs.py $O/old.npz \
      > $O/dump_old.log 2>&1 || { tail -20 $O/dump_old.log; exit 1; }
  DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/${NEW:-libdensityflows_hip.so} timeout -k 10 240 python3 tools/dump_outputs.py $O/new.npz \
      > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
  python3 tools/dump_outputs.py --compare $O/old.npz $O/new.npz | tee $O/compare.txt
  rm -f $O/old.npz $O/new.npz
fi
exec_ab() { bash tools/gpu_ab4.sh "$1"; }
exec_ab "$1"
