set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_forest_gpu.py tests/test_models_gpu.py -x -q > gpurun_out/pytest11.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 200 python scripts/sweep_tiers.py > gpurun_out/sw11.log 2>&1 && grep build gpurun_out/sw11.log && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench11.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/bench11.log
