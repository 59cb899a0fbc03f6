# Forest arena: GPU tests for the forest path, then bench c4 / c8 and phases.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forest_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ar_pytest.log 2>&1 && tail -1 gpurun_out/ar_pytest.log && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/ar_c4.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/ar_c4.log && grep phases gpurun_out/ar_c4.log | cut -c1-600 && \
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cands-per-rank 8 > gpurun_out/ar_c8.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/ar_c8.log && grep phases gpurun_out/ar_c8.log | cut -c1-600
