#!/bin/bash
# round 5: regression large-tier chunk with packed words (<= 3840 rows) -- config 6 sweep
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for ch in 3840 2560 1920 3072; do
  DML_TIER_CHUNK_REG=$ch timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/ch_c6.log 2>&1 || exit 1
  echo "[chunk=$ch] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/ch_c6.log)"
done
done
