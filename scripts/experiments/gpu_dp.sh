set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_data_parallel.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/dp_pytest.log 2>&1 && echo DP_OK && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/all_gpu_pytest.log 2>&1 && tail -2 gpurun_out/all_gpu_pytest.log
