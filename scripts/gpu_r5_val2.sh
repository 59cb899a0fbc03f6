# Round-5 validation 3: every GPU test, smoke, headline bench, LR config 4, GBRT config 6 (+huber variant).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r5v3}
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && tail -1 gpurun_out/${T}_smoke.log && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1 && tail -1 gpurun_out/${T}_bench.log | cut -c1-160 && \
timeout -k 10 400 python -u bench.py --config lr --steps 3 --warmup 1 > gpurun_out/${T}_lr.log 2>&1 && tail -1 gpurun_out/${T}_lr.log | cut -c1-200 && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/${T}_c6.log 2>&1 && grep cv_fits gpurun_out/${T}_c6.log | cut -c1-120 && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 --gb-loss huber > gpurun_out/${T}_c6h.log 2>&1 && grep cv_fits gpurun_out/${T}_c6h.log | cut -c1-120
