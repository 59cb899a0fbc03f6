set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_forest_gpu.py tests/test_models_gpu.py -x -q > gpurun_out/pytest_ab2.log 2>&1 && echo PYTEST_OK && \
for v in old v2_b1 v2_b2 v2_b4; do DML_HIP_LIB=$GRAFT_REPO_ROOT/variants/$v.so timeout -k 10 200 python scripts/sweep_tiers.py > gpurun_out/ab2_$v.log 2>&1 || exit 1; echo "$v $(grep build gpurun_out/ab2_$v.log)"; done && \
DML_HIP_LIB=$GRAFT_REPO_ROOT/variants/v2_b4_prof.so timeout -k 10 200 python scripts/phase_prof.py > gpurun_out/phase_v2.log 2>&1 && grep -v amdgpu gpurun_out/phase_v2.log
