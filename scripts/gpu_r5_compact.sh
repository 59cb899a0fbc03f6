#!/bin/bash
# round 5: compact 3-KB large-tier LDS slices for unit-weight regression builds (boosting)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_models_gpu.py -k "gbrt" tests/test_forest_gpu.py > gpurun_out/cp_tests.log 2>&1; rc=$?; tail -1 gpurun_out/cp_tests.log; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
for v in 0 1; do
  if [ $v = 1 ]; then export DML_LARGE_NO_COMPACT=1; else unset DML_LARGE_NO_COMPACT; fi
  timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/cp_c6.log 2>&1 || exit 1
  echo "[no_compact=$v] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/cp_c6.log)"
done
done
unset DML_LARGE_NO_COMPACT
timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 --gb-loss huber > gpurun_out/cp_c6h.log 2>&1 || exit 1
echo "[huber] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/cp_c6h.log)"
