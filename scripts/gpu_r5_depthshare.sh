#!/bin/bash
# round 5: prefix sharing with nested max_depth (forests, depth-capped predicts) -- tests, then
# config 2 with random_state=0 (sharing on / off)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_prefix_sharing.py tests/test_model_predictor.py tests/test_forest_gpu.py > gpurun_out/ds_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ds_tests.log; [ $rc = 0 ] || exit $rc
for v in 1 0; do
  DML_PREFIX_SHARE=$v timeout -k 10 400 python -u scripts/bench_configs.py --configs 2 --random-state 0 > gpurun_out/ds_c2.log 2>&1 || exit 1
  echo "[c2 rs=0 share=$v] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/ds_c2.log)"
done
