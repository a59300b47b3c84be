#!/bin/bash
# GPU box, round-4 measurement pass: the -m gpu suite, smoke, the driver's bench command
# (and a longer run), every secondary workload, kernel traces (the driver's exact command
# included) and PMC passes (tools/pmc_sets.txt, one counter set per run) of the forward
# and training kernels.  Collected into profiles/ by tools/collect_profiles.py.
# NOPMC=1: everything but the PMC passes; PMCONLY=1: the PMC passes alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4}
mkdir -p $O
python3 -c "import bench; print(bench.source_sha16())" > $O/source_sha16.txt
if [ "${PMCONLY:-0}" != 1 ]; then  # PMCONLY=1: the PMC passes alone (a second call)
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err && \
timeout -k 10 240 python3 bench.py --steps 200 --warmup 50 --cpu-seconds 15 > $O/bench.json 2> $O/bench.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_driver.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --no-cpu > $O/prof.log 2>&1 && \
timeout -k 10 240 python bench.py --config cfg1 --batch 4096 --steps 500 --warmup 100 --cpu-seconds 10 > $O/cfg1_4096.json 2> $O/cfg1_4096.err && \
timeout -k 10 240 python bench.py --config cfg1 --steps 200 --warmup 50 --cpu-seconds 10 > $O/cfg1.json 2> $O/cfg1.err && \
timeout -k 10 240 python bench.py --config cfg4 --steps 20 --warmup 10 --cpu-seconds 15 > $O/cfg4.json 2> $O/cfg4.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg4 -o run -- \
    python3 bench.py --config cfg4 --steps 10 --warmup 3 --no-cpu > $O/prof_cfg4.log 2>&1 && \
timeout -k 10 240 python bench.py --mode nll --steps 100 --warmup 20 > $O/nll.json 2> $O/nll.err && \
timeout -k 10 240 python bench.py --mode train --steps 20 --warmup 5 > $O/train_cfg2.json 2> $O/train_cfg2.err && \
timeout -k 10 300 python bench.py --mode train --config cfg4 --steps 5 --warmup 2 > $O/train_cfg5.json 2> $O/train_cfg5.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t2 -o run -- \
    python3 bench.py --mode train --steps 10 --warmup 3 > $O/prof_t2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t5 -o run -- \
    python3 bench.py --mode train --config cfg4 --steps 3 --warmup 1 > $O/prof_t5.log 2>&1 || exit 1
fi
[ "${NOPMC:-0}" = 1 ] && exit 0
i=0
for cfg in cfg2 cfg4; do
  steps=5; [ $cfg = cfg4 ] && steps=3
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $line --output-format csv -d $O/pmc_${cfg}/p$i -o run -- \
        python3 bench.py --config $cfg --steps $steps --warmup 1 --no-cpu --no-exact --settle-seconds 0 > $O/pmc_${cfg}_p$i.log 2>&1 || exit 1
  done < tools/pmc_sets.txt
done
for cfg in cfg2 cfg4; do
  steps=3; [ $cfg = cfg4 ] && steps=1
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line --output-format csv -d $O/pmct_${cfg}/p$i -o run -- \
        python3 bench.py --mode train --config $cfg --steps $steps --warmup 1 --no-cpu --settle-seconds 0 > $O/pmct_${cfg}_p$i.log 2>&1 || exit 1
  done < tools/pmc_sets.txt
done
