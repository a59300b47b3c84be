# GPU box: the whole -m gpu suite (no -x: every failure is reported), then the
# df_comm NLL bench at one rank.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t
export TMPDIR=/tmp
O=gpurun_out/t
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python bench.py --mode nll --steps 100 --warmup 20 > $O/nll.json 2> $O/nll.err && \
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
