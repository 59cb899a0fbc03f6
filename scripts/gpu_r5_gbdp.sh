#!/bin/bash
# round 5: fused GBRT for deep trees + the row-sharded fused stage (2 ranks sharing the GPU)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_data_parallel.py -m gpu > gpurun_out/r5_gbdp_tests2.log 2>&1
