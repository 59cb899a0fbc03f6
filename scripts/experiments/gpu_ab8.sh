set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/sweep_tiers.py sub_big=0,1 wave_max=128,192,256 > gpurun_out/ab8.log 2>&1; grep build gpurun_out/ab8.log
