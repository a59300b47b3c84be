# GPU box: smoke, the whole GPU test suite, headline bench + rocprofv3 kernel trace, secondary benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/round
export TMPDIR=/tmp
O=gpurun_out/round
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python bench.py --cpu-seconds 12 > $O/bench.json 2> $O/bench.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --no-cpu > $O/prof.log 2>&1 && \
timeout -k 10 240 python bench.py --config cfg4 --steps 20 --warmup 10 --cpu-seconds 12 > $O/cfg4.json 2> $O/cfg4.err && \
timeout -k 10 240 python bench.py --config cfg1 --steps 200 --warmup 50 --no-cpu > $O/cfg1.json 2> $O/cfg1.err && \
timeout -k 10 240 python bench.py --mode nll --steps 100 --warmup 20 > $O/nll.json 2> $O/nll.err && \
timeout -k 10 240 python bench.py --mode train --steps 20 --warmup 5 > $O/train_cfg2.json 2> $O/train_cfg2.err && \
timeout -k 10 300 python bench.py --mode train --config cfg4 --steps 5 --warmup 2 > $O/train_cfg5.json 2> $O/train_cfg5.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t5 -o run -- \
    python3 bench.py --mode train --config cfg4 --steps 2 --warmup 1 > $O/prof_t5.log 2>&1
