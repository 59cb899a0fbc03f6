#!/bin/bash
# round 5: config 2 (RF 64-pt grid) with random_state=0 as ONE run_candidates call: prefix sharing
# nests n_estimators and max_depth (on / off)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 1 0; do
  DML_PREFIX_SHARE=$v timeout -k 10 500 python -u scripts/bench_configs.py --configs 2 --random-state 0 --whole > gpurun_out/ds2_c2.log 2>&1 || exit 1
  echo "[c2 whole rs=0 share=$v] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/ds2_c2.log)"
done
