# Multi-rank rehearsal of bench.py on ONE GPU: ranks share device 0 over gloo (RCCL needs
# one device per rank).  Checks the N>1 code path (sharded synthetic data + all-gather,
# LPT step placement, score all-reduce, max-over-ranks timing); the timings are not
# meaningful (the ranks share one GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export DML_SHARE_DEVICE=1 DML_DIST_BACKEND=gloo DML_HBM_BUDGET_GB=40
timeout -k 10 400 python bench.py --gpus 2 --rows 250000 --steps 2 --warmup 1 --master-port 29611 > gpurun_out/rh2.log 2>&1 && tail -1 gpurun_out/rh2.log | cut -c1-330 && \
timeout -k 10 400 python bench.py --gpus 4 --rows 250000 --steps 1 --warmup 1 --master-port 29612 > gpurun_out/rh4.log 2>&1 && tail -1 gpurun_out/rh4.log | cut -c1-330
