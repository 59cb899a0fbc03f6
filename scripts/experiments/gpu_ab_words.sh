set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forest_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/words_pytest.log 2>&1 && echo PYTEST_OK && \
DML_ROW_WORDS_OFF=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/words0.log 2>&1 && tail -1 gpurun_out/words0.log | cut -c1-200 && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/words1.log 2>&1 && tail -1 gpurun_out/words1.log | cut -c1-200
