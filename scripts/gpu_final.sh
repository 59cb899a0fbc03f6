# Round-end check: GPU test tier, smoke, headline bench, whole 256 x 5 grid on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/fin_pytest.log 2>&1 && tail -1 gpurun_out/fin_pytest.log && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 && tail -1 gpurun_out/fin_smoke.log && \
timeout -k 10 300 python bench.py > gpurun_out/fin_bench.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/fin_bench.log && \
timeout -k 10 600 python bench.py --steps 16 --warmup 1 --cands-per-rank 16 > gpurun_out/fin_full.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/fin_full.log
