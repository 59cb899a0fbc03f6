set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/ -m gpu -x -q > gpurun_out/pytest5.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench5_n1.log 2>&1 && echo BENCH_OK
