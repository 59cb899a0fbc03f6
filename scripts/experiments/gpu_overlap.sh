set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forest_gpu.py -x -q --timeout 120 --timeout-method thread -k "overlapped or match_cpu" > gpurun_out/ov_pytest.log 2>&1 && tail -1 gpurun_out/ov_pytest.log && \
timeout -k 10 600 python bench.py --steps 16 --warmup 1 --cands-per-rank 16 > gpurun_out/ov_full.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/ov_full.log && grep phases gpurun_out/ov_full.log | cut -c1-600 && \
timeout -k 10 400 python scripts/bench_configs.py --configs 2 > gpurun_out/ov_cfg2.log 2>&1 && grep '^{' gpurun_out/ov_cfg2.log
