set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_models_gpu.py -x -q > gpurun_out/pytest7.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 400 python scripts/bench_configs.py --configs 2,5 > gpurun_out/configs25.log 2>&1 && echo C25_OK && \
timeout -k 10 400 python scripts/bench_configs.py --configs 4 --lr-rows 2000000 > gpurun_out/config4.log 2>&1 && echo C4_OK
