set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/sweep_tiers.py kg_wave=4 > gpurun_out/sweep6a.log 2>&1 && grep -v amdgpu.ids gpurun_out/sweep6a.log | tail -1 && \
DML_HIP_LIB=$GRAFT_REPO_ROOT/variants/libdml_hip_kg8.so timeout -k 10 400 python -u scripts/sweep_tiers.py kg_wave=4,6,8 > gpurun_out/sweep6b.log 2>&1 && grep -v amdgpu.ids gpurun_out/sweep6b.log | tail -3
