# Round validation on one GPU: GPU tests, smoke, headline bench, whole-grid bench, e2e bench.
#   gpurun --timeout 1200 -- bash scripts/gpu_validate.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-v}
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && tail -1 gpurun_out/${T}_smoke.log && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1 && tail -1 gpurun_out/${T}_bench.log | cut -c1-160 && \
timeout -k 10 400 python -u bench.py --cands-per-rank 16 --steps 16 --warmup 1 > gpurun_out/${T}_fullgrid.log 2>&1 && tail -1 gpurun_out/${T}_fullgrid.log | cut -c1-160 && \
timeout -k 10 600 python -u bench.py --e2e > gpurun_out/${T}_e2e.log 2>&1 && tail -1 gpurun_out/${T}_e2e.log | cut -c1-200
