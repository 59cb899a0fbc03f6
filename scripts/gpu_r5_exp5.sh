# Round-5 batch 5: LR skips column tiles of stopped fits (C-ordered column layout).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $PYT -m gpu tests/test_models_gpu.py tests/test_lr_device_solver.py tests/test_lr_config4_fidelity.py -k "lr or logistic or Logistic" > gpurun_out/e7_tests.log 2>&1; rc=$?; tail -2 gpurun_out/e7_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config lr --steps 3 --warmup 1 > gpurun_out/e7_lrbench.log 2>&1 && tail -1 gpurun_out/e7_lrbench.log | cut -c1-220 && grep phases gpurun_out/e7_lrbench.log | cut -c1-300 && \
DML_LR_SKIP_DONE=0 timeout -k 10 400 python -u bench.py --config lr --steps 3 --warmup 1 > gpurun_out/e7_lrbench_noskip.log 2>&1 && tail -1 gpurun_out/e7_lrbench_noskip.log | cut -c1-220
