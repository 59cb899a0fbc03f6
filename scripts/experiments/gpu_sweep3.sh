set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/sweep_tiers.py wave_max=512 block_max=131072,262144,1048576 chunk=8192,16384 > gpurun_out/sweep3.log 2>&1 && grep -v amdgpu.ids gpurun_out/sweep3.log | tail -14
