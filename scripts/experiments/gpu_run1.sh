set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_forest_gpu.py -x -q > gpurun_out/pytest1.log 2>&1 && echo PYTEST_OK
timeout -k 10 240 python scripts/gbench_forest.py 200000 50 10 5 > gpurun_out/gbench_small.log 2>&1 && echo SMALL_OK && \
timeout -k 10 300 python scripts/gbench_forest.py 1000000 100 20 5 > gpurun_out/gbench_1m.log 2>&1 && echo BIG_OK
