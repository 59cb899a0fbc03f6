set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python scripts/bench_configs.py --configs 2,5 > gpurun_out/cfg25b.log 2>&1 && grep '^{' gpurun_out/cfg25b.log && \
timeout -k 10 600 python scripts/bench_configs.py --configs 4 --lr-rows 10000000 > gpurun_out/cfg4b.log 2>&1 && grep '^{' gpurun_out/cfg4b.log
