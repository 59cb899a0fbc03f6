set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python scripts/sweep_tiers.py > gpurun_out/ab7.log 2>&1 && grep build gpurun_out/ab7.log && \
timeout -k 10 200 python scripts/sweep_tiers.py sub_big=0 > gpurun_out/ab7b.log 2>&1 && grep build gpurun_out/ab7b.log && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench7.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/bench7.log
