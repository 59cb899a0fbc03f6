set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forest_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pad_pytest.log 2>&1 && echo PYTEST_OK && \
DML_XB_PAD=0 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/pad0.log 2>&1 && tail -1 gpurun_out/pad0.log | cut -c1-200 && \
DML_XB_PAD=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/pad1.log 2>&1 && tail -1 gpurun_out/pad1.log | cut -c1-200
