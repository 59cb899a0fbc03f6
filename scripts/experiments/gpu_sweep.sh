set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python scripts/sweep_tiers.py kg_wave=2,4,8 kg_block=8,16,32 > gpurun_out/sweep1.log 2>&1 && echo S1_OK && \
timeout -k 10 500 python scripts/sweep_tiers.py wave_max=128,256 block_max=4096,16384,65536 > gpurun_out/sweep2.log 2>&1 && echo S2_OK
