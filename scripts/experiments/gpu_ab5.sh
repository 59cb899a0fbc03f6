set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_forest_gpu.py tests/test_models_gpu.py -x -q > gpurun_out/pytest_ab5.log 2>&1 && echo PYTEST_OK && \
for v in v4_nt256 v5; do DML_HIP_LIB=$GRAFT_REPO_ROOT/variants/$v.so timeout -k 10 200 python scripts/sweep_tiers.py > gpurun_out/ab5_$v.log 2>&1 || exit 1; echo "$v $(grep build gpurun_out/ab5_$v.log)"; done
