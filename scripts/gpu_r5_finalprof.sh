#!/bin/bash
# round 5 final: rocprofv3 kernel stats of the headline bench and GBRT config 6 at HEAD
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp_bench -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/fp_bench.log 2>&1 || exit 1
f=$(find gpurun_out/fp_bench -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/fp_bench_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp_c6 -- python3 scripts/bench_configs.py --configs 6 > gpurun_out/fp_c6.log 2>&1 || exit 1
f=$(find gpurun_out/fp_c6 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/fp_c6_kernel_stats.csv
python3 scripts/gaps.py gpurun_out/fp_c6 20 0.3 > gpurun_out/fp_c6_gaps.txt 2>&1 || true
find gpurun_out/fp_bench gpurun_out/fp_c6 -name "*kernel_trace.csv" -delete
grep '^{' gpurun_out/fp_bench.log | cut -c1-120
grep -o '"cv_fits_per_s[^,]*' gpurun_out/fp_c6.log
head -3 gpurun_out/fp_c6_gaps.txt
