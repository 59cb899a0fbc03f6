#!/bin/bash
# round 5: boosting lanes 1 / 2 in steady state -- config 6 repeated 4x in one process
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
run() { timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/cl.log 2>&1 || exit 1; echo "[$1] $(grep -o 'repeat [0-9]: [0-9.]* s' gpurun_out/cl.log | tr '\n' ' ') last: $(grep -o '"seconds": [0-9.]*' gpurun_out/cl.log | head -1)"; }
for rep in 1 2; do
DML_C6_WARMUP=0 DML_C6_REPEAT=4 DML_GB_LANES=1 run "lanes=1"
DML_C6_WARMUP=0 DML_C6_REPEAT=4 DML_GB_LANES=2 run "lanes=2"
DML_C6_WARMUP=0 DML_C6_REPEAT=4 DML_GB_LANES=3 run "lanes=3"
done
