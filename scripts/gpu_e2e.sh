# End-to-end job path on one GPU: bench --e2e through the LocalRunner and through the
# cluster DistributedRunner (world-1 RCCL group), config 5 through the DistributedRunner,
# and the kernel bench for comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/e2e_kbench.log 2>&1 && tail -1 gpurun_out/e2e_kbench.log | cut -c1-140 && \
timeout -k 10 900 python -u bench.py --e2e > gpurun_out/e2e_local.log 2>&1 && tail -1 gpurun_out/e2e_local.log && \
DML_FORCE_PG=1 MASTER_PORT=29601 timeout -k 10 900 python -u bench.py --e2e > gpurun_out/e2e_dist.log 2>&1 && tail -1 gpurun_out/e2e_dist.log && \
DML_FORCE_PG=1 MASTER_PORT=29602 timeout -k 10 600 python -u scripts/bench_configs.py --configs 5 > gpurun_out/cfg5_dist.log 2>&1 && tail -1 gpurun_out/cfg5_dist.log
