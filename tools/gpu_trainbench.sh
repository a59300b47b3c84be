set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --mode train --steps 10 --warmup 2 > gpurun_out/train_cfg2.json 2> gpurun_out/train_cfg2.err && \
timeout -k 10 200 python bench.py --mode train --config cfg1 --batch 65536 --steps 20 --warmup 3 > gpurun_out/train_cfg1.json 2> gpurun_out/train_cfg1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run -- python bench.py --mode train --steps 5 --warmup 1 > gpurun_out/train_prof.log 2>&1
