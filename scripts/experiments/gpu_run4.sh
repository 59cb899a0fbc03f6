set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_forest_gpu.py -x -q > gpurun_out/pytest4.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python scripts/gbench_forest.py 1000000 100 20 5 > gpurun_out/gbench_1m.log 2>&1 && echo GB_OK && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_n1.log 2>&1 && echo BENCH_OK
