#!/bin/bash
# round 5: back-to-back boosting jobs -- repeated runs in one process, lanes / root cache toggles
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
run() { timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/cw3.log 2>&1 || exit 1; echo "[$1] $(grep -o 'repeat [0-9]: [0-9.]* s' gpurun_out/cw3.log | tr '\n' ' ') last: $(grep -o '"seconds": [0-9.]*' gpurun_out/cw3.log | head -1)"; }
DML_C6_WARMUP=0 DML_C6_REPEAT=3 run "x3 same job"
DML_C6_WARMUP=1 DML_GB_LANES=1 run "warm lanes=1"
DML_C6_WARMUP=0 DML_GB_LANES=1 run "cold lanes=1"
DML_C6_WARMUP=1 DML_GB_ROOT_CACHE=0 run "warm nocache"
DML_C6_WARMUP=0 DML_GB_ROOT_CACHE=0 run "cold nocache"
