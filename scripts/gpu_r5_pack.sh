#!/bin/bash
# round 5: packed count | w yq LDS words for unit-weight regression builds -- tests, then config 6
# packed vs unpacked (DML_LARGE_NO_PACK=1), huber variant, depth profile
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_models_gpu.py tests/test_forest_gpu.py tests/test_prefix_sharing.py tests/test_data_parallel.py > gpurun_out/pk_tests.log 2>&1; rc=$?; tail -1 gpurun_out/pk_tests.log; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
for v in 0 1; do
  if [ $v = 1 ]; then export DML_LARGE_NO_PACK=1; else unset DML_LARGE_NO_PACK; fi
  timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/pk_c6.log 2>&1 || exit 1
  echo "[no_pack=$v] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/pk_c6.log)"
done
done
unset DML_LARGE_NO_PACK
timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 --gb-loss huber > gpurun_out/pk_c6h.log 2>&1 || exit 1
echo "[huber] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/pk_c6h.log)"
timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 --gb-loss squared_error > gpurun_out/pk_c6s.log 2>&1 || exit 1
echo "[squared_error] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/pk_c6s.log)"
