set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_wide.log 2>&1 ; \
timeout -k 10 120 python bench.py --config cfg4 --steps 5 --warmup 2 --no-cpu > gpurun_out/cfg4_wide.json 2>/dev/null && \
DF_NO_WIDE=1 timeout -k 10 120 python bench.py --config cfg4 --steps 5 --warmup 2 --no-cpu > gpurun_out/cfg4_gen.json 2>/dev/null
