#!/bin/bash
# round 5: large-tier feature group width for boosting with compact LDS slices (3 KB / feature:
# 16 -> 3 workgroups per CU, 13 -> 4, 10 -> 5)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for kg in 16 15 13 12 10; do
  DML_TIER_KG_LARGE_REG=$kg timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/kg_c6.log 2>&1 || exit 1
  echo "[kg=$kg] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/kg_c6.log)"
done
done
