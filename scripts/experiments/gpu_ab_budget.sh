set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bud055.log 2>&1 && grep -h "phases\|metric" gpurun_out/bud055.log | cut -c1-330 && \
DML_HBM_FRACTION=0.8 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bud08.log 2>&1 && grep -h "phases\|metric" gpurun_out/bud08.log | cut -c1-330
