#!/bin/bash
# round 5: root-hist microbench with the count atomic and the packed (count | w yq) variant
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/micro_root_hist.bin 1000000 100 > gpurun_out/rh_micro2.txt 2>&1; rc=$?; cat gpurun_out/rh_micro2.txt; exit $rc
