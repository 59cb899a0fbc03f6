#!/bin/bash
# round 5: exact n_estimators prefix sharing -- GPU tests, then configs 2 and 6 with a fixed
# random_state, sharing on vs off (DML_PREFIX_SHARE=0), and config 2 as shipped (random_state None)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_prefix_sharing.py > gpurun_out/px_tests.log 2>&1 || exit 1
tail -1 gpurun_out/px_tests.log
for v in "1 0" "0 0"; do
  set -- $v
  DML_PREFIX_SHARE=$1 timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 --random-state $2 > gpurun_out/px_c6.log 2>&1 || exit 1
  echo "[c6 rs=$2 share=$1] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/px_c6.log) $(grep -o '"best_mean_cv[^,]*' gpurun_out/px_c6.log)"
done
for v in "1 0" "0 0"; do
  set -- $v
  DML_PREFIX_SHARE=$1 timeout -k 10 400 python -u scripts/bench_configs.py --configs 2 --random-state $2 > gpurun_out/px_c2.log 2>&1 || exit 1
  echo "[c2 rs=$2 share=$1] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/px_c2.log)"
done
timeout -k 10 400 python -u scripts/bench_configs.py --configs 2 > gpurun_out/px_c2.log 2>&1 || exit 1
echo "[c2 rs=None] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/px_c2.log)"
