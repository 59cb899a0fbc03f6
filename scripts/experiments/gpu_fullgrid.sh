# Whole 256-pt grid on one GPU (ground truth for the sampled per-step metric), then the
# default bench and a larger per-step batch, all with the low-discrepancy candidate order.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/fg_c4.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/fg_c4.log && \
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cands-per-rank 8 > gpurun_out/fg_c8.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/fg_c8.log && \
timeout -k 10 600 python bench.py --steps 16 --warmup 1 --cands-per-rank 16 > gpurun_out/fg_full.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/fg_full.log
