set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
DML_HIP_LIB=$GRAFT_REPO_ROOT/variants/v8_prof.so timeout -k 10 200 python scripts/phase_prof.py > gpurun_out/phase_v7.log 2>&1; grep -v amdgpu gpurun_out/phase_v7.log | tail -3
