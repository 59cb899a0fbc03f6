#!/bin/bash
# round 5: boosting large tier -- feature-major gathers only above 1/k of the rows (row-major
# lines below); k = 0: feature-major everywhere (default)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for k in 0 2 4 8 16 1000000000; do
  DML_LARGE_FM_DIV=$k timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/fm_c6.log 2>&1 || exit 1
  echo "[fm_div=$k] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/fm_c6.log)"
done
done
