set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_forest_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pk_pytest.log 2>&1 && tail -1 gpurun_out/pk_pytest.log && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/pk_bench.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/pk_bench.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pkprof -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/pk_prof.log 2>&1 && python scripts/summarize_prof.py /tmp/pkprof > gpurun_out/pk_stats.txt 2>&1 && head -8 gpurun_out/pk_stats.txt | cut -c1-140
