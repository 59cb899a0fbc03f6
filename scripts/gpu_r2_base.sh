# Round-2 baseline: gpu tests, driver-shaped bench (20 steps / 5 warmup), rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b2_pytest.log 2>&1; echo "PYTEST rc=$?"; tail -2 gpurun_out/b2_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b2_bench.log 2>&1 && tail -1 gpurun_out/b2_bench.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/b2_prof -o run -- python bench.py --steps 4 --warmup 1 > gpurun_out/b2_prof.log 2>&1 && echo PROF_OK
