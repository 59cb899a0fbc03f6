set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_forest_gpu.py -x -q > gpurun_out/pytest3.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_n1.log 2>&1 && echo BENCH_OK && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rf2 -o run -- python bench.py --steps 1 --warmup 0 > gpurun_out/prof_rf2.log 2>&1 && echo PROF_OK
