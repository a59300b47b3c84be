set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_train.py -x -q -rA > gpurun_out/pytest_train.log 2>&1
