#!/bin/bash
# round 5: GPU busy of config 6 in steady state (3rd of 3 back-to-back jobs; last ~30 % of the trace)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DML_C6_WARMUP=0 DML_C6_REPEAT=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cb_prof -- python3 scripts/bench_configs.py --configs 6 > gpurun_out/cb_c6.log 2>&1 || exit 1
grep -o 'repeat [0-9]: [0-9.]* s' gpurun_out/cb_c6.log | tr '\n' ' '; grep -o '"seconds": [0-9.]*' gpurun_out/cb_c6.log | head -1
python3 scripts/gaps.py gpurun_out/cb_prof 20 0.72 | head -8
find gpurun_out/cb_prof -name "*kernel_trace.csv" -delete
