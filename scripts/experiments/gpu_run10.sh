set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_forest_gpu.py tests/test_models_gpu.py -x -q > gpurun_out/pytest10.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench10.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/bench10.log && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof10 -o b -- python bench.py --steps 1 --warmup 1 > gpurun_out/prof10.log 2>&1 && echo PROF_OK
