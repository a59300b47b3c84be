# GPU box: smoke, the whole GPU test suite, headline bench, secondary benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --cpu-seconds 12 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 240 python bench.py --config cfg4 --steps 5 --warmup 2 --cpu-seconds 12 > gpurun_out/cfg4.json 2> gpurun_out/cfg4.err && \
timeout -k 10 240 python bench.py --mode nll --steps 20 --warmup 3 > gpurun_out/nll.json 2> gpurun_out/nll.err && \
timeout -k 10 240 python bench.py --mode train --steps 10 --warmup 2 > gpurun_out/train_cfg2.json 2> gpurun_out/train_cfg2.err && \
timeout -k 10 300 python bench.py --mode train --config cfg4 --steps 3 --warmup 1 > gpurun_out/train_cfg5.json 2> gpurun_out/train_cfg5.err
