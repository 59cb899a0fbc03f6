# One GPU call: gpu tests, smoke, headline bench, rocprof kernel stats of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/chk_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/chk_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/chk_bench.log 2>&1 && tail -1 gpurun_out/chk_bench.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/chk_prof -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/chk_prof.log 2>&1 && echo PROF_OK
