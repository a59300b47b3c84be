#!/bin/bash
# GPU box: reproduce the driver's bench command and look at its clock.
#   1. the GPU suite (parity) on the current build
#   2. the driver's exact command (--steps 20 --warmup 5), twice, and once with per-step times
#   3. a long run (200 / 50) with per-step times
#   4. a kernel trace of exactly the driver's command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-clk}
mkdir -p $O
python3 -c "import bench; print(bench.source_sha16())" > $O/source_sha16.txt
if [ "${NOTEST:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
fi
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver1.json 2> $O/driver1.err && \
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/driver2.json 2> $O/driver2.err && \
DF_BENCH_STEPLOG=1 timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/driver_steplog.json 2> $O/driver_steplog.err && \
DF_BENCH_STEPLOG=1 timeout -k 10 240 python3 bench.py --steps 200 --warmup 50 --no-cpu > $O/long_steplog.json 2> $O/long_steplog.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_driver.log 2>&1 || exit 1
