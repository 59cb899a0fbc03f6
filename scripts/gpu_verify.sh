# One GPU call: GPU test tier, smoke, headline bench (1 GPU).
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/verify_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/verify_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/verify_bench.log 2>&1 && tail -1 gpurun_out/verify_bench.log
