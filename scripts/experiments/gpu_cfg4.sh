set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cfg4_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 600 python scripts/bench_configs.py --configs 4 --lr-rows 10000000 > gpurun_out/cfg4.log 2>&1 && grep cv_fits gpurun_out/cfg4.log
