#!/bin/bash
# GPU box: LDS bank conflicts and MFMA busy (or the counter sets in $SETS, ';'-separated)
# of one workload under several library builds, one PMC pass per set and build.
#   tools/gpu_conflicts.sh <tag> "<bench args>" <kernel substring> <lib> [<lib> ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; ARGS=$2; K=$3
shift 3
mkdir -p $O
for lib in "$@"; do
  IFS=';' read -ra SETL <<< "${SETS:-SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE;SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES}"
  for set in "${SETL[@]}"; do
    n=$(echo $set | cut -c1-12 | tr ' ' '_')
    DENSITYFLOWS_HIP_LIB=densityflows.jl_amd/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv \
        -d $O/${lib%.so}/p_$n -o run -- python3 bench.py $ARGS --no-cpu --no-exact --settle-seconds 0 > $O/${lib%.so}_$n.log 2>&1 || exit 1
  done
  echo "== $lib" >> $O/summary.txt
  python3 tools/pmc_summary.py $1/${lib%.so} "$K" >> $O/summary.txt
done
cat $O/summary.txt
