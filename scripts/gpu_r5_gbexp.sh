#!/bin/bash
# round 5: GBRT config 6 build lanes 1-4, and a deep-tree variant (max_depth 8 / 10) fused vs torch stage
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for l in 1 2 3 4; do
  DML_GB_LANES=$l timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/gbx_c6.log 2>&1 || exit 1
  echo "[lanes=$l] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/gbx_c6.log)"
done
for f in 1 0; do
  DML_GB_FUSED=$f timeout -k 10 400 python -u scripts/bench_configs.py --configs 6 --gb-depths 8,10 --gb-estimators 20,40 > gpurun_out/gbx_deep.log 2>&1 || exit 1
  echo "[deep fused=$f] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/gbx_deep.log) $(grep -o '"best_mean_cv[^,]*' gpurun_out/gbx_deep.log)"
done
