set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_forest_gpu.py -q -k "wave_primitives or kw0-2 or kw0-1" > gpurun_out/pytest_dbg.log 2>&1; echo rc=$?
