#!/bin/bash
# round 5: config 6 with an untimed warmup fit (default) vs without (DML_C6_WARMUP=0), interleaved
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do
for w in 1 0; do
  DML_C6_WARMUP=$w timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/cw_c6.log 2>&1 || exit 1
  echo "[warmup=$w] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/cw_c6.log)"
done
done
timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 --gb-loss huber > gpurun_out/cw_c6h.log 2>&1 || exit 1
echo "[huber warmup=1] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/cw_c6h.log)"
