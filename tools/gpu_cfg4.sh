set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -x -q > gpurun_out/pytest_cfg4.log 2>&1 && \
timeout -k 10 120 python bench.py --config cfg4 --batch 262144 --steps 5 --warmup 2 --no-cpu > gpurun_out/cfg4.json 2>/dev/null && \
timeout -k 10 200 python bench.py --mode train --config cfg4 --batch 262144 --steps 3 --warmup 1 > gpurun_out/train_cfg5.json 2>/dev/null
