# One GPU call: predicted weak-scaling efficiency of bench.py placements, then the 1-GPU bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/scaling_sim.py --world 2,4,8 --steps 2 > gpurun_out/scaling_sim.log 2>&1 && cat gpurun_out/scaling_sim.log && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/sim_bench.log 2>&1 && tail -1 gpurun_out/sim_bench.log
