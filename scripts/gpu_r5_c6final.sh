#!/bin/bash
# round 5: config 6 at the new defaults (3 build lanes, lane streams reused, untimed warmup fit) vs cold
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_models_gpu.py -k gbrt tests/test_data_parallel.py > gpurun_out/cf_tests.log 2>&1; rc=$?; tail -1 gpurun_out/cf_tests.log; [ $rc = 0 ] || exit $rc
for rep in 1 2 3; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/cf_c6.log 2>&1 || exit 1
  echo "[warm, lanes 3] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/cf_c6.log)"
  DML_C6_WARMUP=0 timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/cf_c6c.log 2>&1 || exit 1
  echo "[cold, lanes 3] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/cf_c6c.log)"
done
timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 --gb-loss huber > gpurun_out/cf_c6h.log 2>&1 || exit 1
echo "[huber warm] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/cf_c6h.log)"
