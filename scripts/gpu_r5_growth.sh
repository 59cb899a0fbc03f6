#!/bin/bash
# round 5: whole-histogram buffers grown 2x (fewer hipFree device syncs) -- config 6 x3 + huber, gaps
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/gr_c6.log 2>&1 || exit 1
  echo "[c6] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/gr_c6.log)"
done
timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 --gb-loss huber > gpurun_out/gr_c6h.log 2>&1 || exit 1
echo "[huber] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/gr_c6h.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gr_prof -- python3 scripts/bench_configs.py --configs 6 > gpurun_out/gr_c6p.log 2>&1 || exit 1
python3 scripts/gaps.py gpurun_out/gr_prof 20 0.3 > gpurun_out/gr_gaps.txt 2>&1 || true
find gpurun_out/gr_prof -name "*kernel_trace.csv" -delete
head -6 gpurun_out/gr_gaps.txt
