#!/bin/bash
# round 5: host-side profile of a boosting run with stumps (the per-stage host cost)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m cProfile -o gpurun_out/hp.prof scripts/bench_configs.py --configs 6 --gb-depths 1 --gb-estimators 100,200 > gpurun_out/hp_c6.log 2>&1 || exit 1
grep -o '"cv_fits_per_s[^,]*' gpurun_out/hp_c6.log
python3 -c "
import pstats
p = pstats.Stats('gpurun_out/hp.prof')
p.sort_stats('cumulative').print_stats(45)
" 2>&1 | tail -50
