#!/bin/bash
# round 5: balanced regression feature rounds (default) vs fixed 16-wide rounds
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_models_gpu.py tests/test_forest_gpu.py tests/test_prefix_sharing.py > gpurun_out/kb_tests.log 2>&1; rc=$?; tail -1 gpurun_out/kb_tests.log; [ $rc = 0 ] || exit $rc
for rep in 1 2 3; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/kb_c6.log 2>&1 || exit 1
  echo "[balanced] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/kb_c6.log)"
done
timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 --gb-loss huber > gpurun_out/kb_c6h.log 2>&1 || exit 1
echo "[huber balanced] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/kb_c6h.log)"
