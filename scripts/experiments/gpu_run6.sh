set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_models_gpu.py -x -q > gpurun_out/pytest6.log 2>&1 && echo PYTEST_OK
