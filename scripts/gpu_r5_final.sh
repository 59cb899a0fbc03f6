#!/bin/bash
# round 5 final validation: every GPU test, smoke, headline bench, whole grid, e2e, LR config 4,
# GBRT config 6 (+ huber), config 2 with random_state (prefix sharing)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r5f}
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && tail -1 gpurun_out/${T}_smoke.log && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1 && tail -1 gpurun_out/${T}_bench.log | cut -c1-160 && \
timeout -k 10 400 python -u bench.py --cands-per-rank 16 --steps 16 --warmup 1 > gpurun_out/${T}_fullgrid.log 2>&1 && tail -1 gpurun_out/${T}_fullgrid.log | cut -c1-160 && \
timeout -k 10 600 python -u bench.py --e2e > gpurun_out/${T}_e2e.log 2>&1 && tail -1 gpurun_out/${T}_e2e.log | cut -c1-200 && \
timeout -k 10 400 python -u bench.py --config lr --steps 3 --warmup 1 > gpurun_out/${T}_lr.log 2>&1 && tail -1 gpurun_out/${T}_lr.log | cut -c1-200 && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/${T}_c6.log 2>&1 && grep -o '"cv_fits_per_s[^,]*' gpurun_out/${T}_c6.log && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 --gb-loss huber > gpurun_out/${T}_c6h.log 2>&1 && grep -o '"cv_fits_per_s[^,]*' gpurun_out/${T}_c6h.log && \
timeout -k 10 400 python -u scripts/bench_configs.py --configs 2 --random-state 0 --whole > gpurun_out/${T}_c2rs.log 2>&1 && grep -o '"cv_fits_per_s[^,]*' gpurun_out/${T}_c2rs.log
