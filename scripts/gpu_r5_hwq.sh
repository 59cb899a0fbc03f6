#!/bin/bash
# round 5: hardware queues per process (GPU_MAX_HW_QUEUES, box default 4) vs the builder's streams
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/hq_bench.log 2>&1 || exit 1
  echo "[hwq=$q] bench $(grep -o '"value": [0-9.]*' gpurun_out/hq_bench.log | head -1)"
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/hq_c6.log 2>&1 || exit 1
  echo "[hwq=$q] c6 $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/hq_c6.log)"
done
