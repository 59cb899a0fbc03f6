#!/bin/bash
# round 5: boosting large-tier histogram cost by tree depth (kernel stats for depth 1 / 3 / 5 grids)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for dep in 1 2 3 4 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dp_prof$dep -- python3 scripts/bench_configs.py --configs 6 --gb-depths $dep --gb-estimators 100,200 > gpurun_out/dp_c6.log 2>&1 || exit 1
  f=$(find gpurun_out/dp_prof$dep -name "*kernel_stats.csv" | head -1)
  echo "depth $dep $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/dp_c6.log)"
  python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:6]:
    print('   ', r['Name'][:44], r['Calls'], round(float(r['TotalDurationNs'])/1e6,1), 'ms')"
  find gpurun_out/dp_prof$dep -name "*kernel_trace.csv" -delete
done
