#!/bin/bash
# round 5: boosting tests, then A/B of the whole-histogram buffer growth (2x vs the old 1.25x), config 6
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_models_gpu.py -k gbrt tests/test_prefix_sharing.py > gpurun_out/ga_tests.log 2>&1; rc=$?; tail -1 gpurun_out/ga_tests.log; [ $rc = 0 ] || exit $rc
L=cs230_distributed_machine_learning_amd/lib
for rep in 1 2 3; do
for v in new g125; do
  if [ $v = new ]; then lib=$L/libdml_hip.so; else lib=$L/libdml_hip_$v.so; fi
  DML_HIP_LIB=$lib timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/ga_c6.log 2>&1 || exit 1
  echo "[$v] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/ga_c6.log)"
done
done
