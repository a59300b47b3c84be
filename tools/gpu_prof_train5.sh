set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_t5 -o run -- python bench.py --mode train --config cfg4 --batch 262144 --steps 2 --warmup 1 > gpurun_out/prof_t5.log 2>&1
