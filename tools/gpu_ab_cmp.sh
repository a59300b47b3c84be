#!/bin/bash
# GPU box: bitwise comparison of a variant build against the in-tree build, its -m gpu
# suite, then the interleaved A/B bench (tools/gpu_ab.sh).
#   tools/gpu_ab_cmp.sh <tag> <variant lib> "<bench args>" [more libs...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; O=gpurun_out/$1; V=$2; ARGS=$3; shift 3
mkdir -p $O
timeout -k 10 300 python3 tools/dump_outputs.py $O/base.npz > $O/dump_base.log 2>&1 && \
DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$V timeout -k 10 300 python3 tools/dump_outputs.py $O/var.npz > $O/dump_var.log 2>&1 || exit 1
python3 tools/dump_outputs.py --compare $O/base.npz $O/var.npz > $O/compare.txt 2>&1; cat $O/compare.txt
TESTLIB=$V bash tools/gpu_ab.sh $TAG "$ARGS" libdensityflows_hip.so $V "$@"
