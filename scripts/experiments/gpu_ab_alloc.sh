# Where does a forest batch spend time outside the build?  Allocation churn A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cands-per-rank 8 > gpurun_out/al_c8.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/al_c8.log && grep phases gpurun_out/al_c8.log | cut -c1-700 && \
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cands-per-rank 8 > gpurun_out/al_c8x.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/al_c8x.log && grep phases gpurun_out/al_c8x.log | cut -c1-700
