#!/bin/bash
# round 5: boosting root-histogram microbenchmark (atomics vs bin-sorted segmented sums) and
# the production root cost (config 6 grid with stumps: every stage is one root level)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./scripts/micro_root_hist.bin 1000000 100 > gpurun_out/rh_micro.txt 2>&1; rc=$?; cat gpurun_out/rh_micro.txt; [ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rh_prof -- python3 scripts/bench_configs.py --configs 6 --gb-depths 1 --gb-estimators 100,200 > gpurun_out/rh_c6.log 2>&1 || exit 1
grep -o '"cv_fits_per_s[^,]*' gpurun_out/rh_c6.log
f=$(find gpurun_out/rh_prof -name "*kernel_stats.csv" | head -1)
head -8 "$f" | cut -d, -f1-4
find gpurun_out/rh_prof -name "*kernel_trace.csv" -delete
