set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/sweep_tiers.py kg_block=8,12,16 kg_wave=2,4 > gpurun_out/sweep4.log 2>&1 && grep -v amdgpu.ids gpurun_out/sweep4.log | tail -7 && \
timeout -k 10 300 python -u scripts/sweep_tiers.py sub_max=32,48,64 > gpurun_out/sweep5.log 2>&1 && grep -v amdgpu.ids gpurun_out/sweep5.log | tail -3
