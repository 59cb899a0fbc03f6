# Round-5 batch 12: LR v4 forward (256 x 256): tests, kernel bench, config-4 bench v4 vs v3.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_models_gpu.py tests/test_lr_device_solver.py tests/test_lr_config4_fidelity.py -k "lr or logistic or Logistic" > gpurun_out/e17_tests.log 2>&1; rc=$?; tail -2 gpurun_out/e17_tests.log; [ $rc = 0 ] || exit $rc
for v in 1 0; do
  DML_LR_V4=$v timeout -k 10 200 python -u scripts/lr_kernel_bench.py 10000000 1000 2560 > gpurun_out/e17_lrk_v4$v.log 2>&1 || exit 1
  echo "v4=$v $(tail -1 gpurun_out/e17_lrk_v4$v.log)"
done
DML_LR_V4=1 timeout -k 10 400 python -u bench.py --config lr --steps 3 --warmup 1 > gpurun_out/e17_lr_v4.log 2>&1 && tail -1 gpurun_out/e17_lr_v4.log | cut -c1-200
