#!/bin/bash
# round 5: k_hist_large time of config 6, packed vs unpacked words
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1; do
  if [ $v = 1 ]; then export DML_LARGE_NO_PACK=1; else unset DML_LARGE_NO_PACK; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pp_prof$v -- python3 scripts/bench_configs.py --configs 6 > gpurun_out/pp_c6.log 2>&1 || exit 1
  f=$(find gpurun_out/pp_prof$v -name "*kernel_stats.csv" | head -1)
  echo "no_pack=$v $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/pp_c6.log)"
  python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:4]:
    print('   ', r['Name'][:44], r['Calls'], round(float(r['TotalDurationNs'])/1e6,1), 'ms')"
  find gpurun_out/pp_prof$v -name "*kernel_trace.csv" -delete
done
