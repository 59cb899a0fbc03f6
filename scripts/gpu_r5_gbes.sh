#!/bin/bash
# round 5: fused boosting stage with early stopping on the percentile losses
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_models_gpu.py -k "gbrt_fused" > gpurun_out/es_tests.log 2>&1; rc=$?; tail -3 gpurun_out/es_tests.log; exit $rc
