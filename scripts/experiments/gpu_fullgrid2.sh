set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cands-per-rank 16 > gpurun_out/fg2_c16.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/fg2_c16.log && \
timeout -k 10 600 python bench.py --steps 16 --warmup 1 --cands-per-rank 16 > gpurun_out/fg2_full.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/fg2_full.log && grep phases gpurun_out/fg2_full.log | cut -c1-600
