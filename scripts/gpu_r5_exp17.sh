# Round-5 batch 17: GBRT config 6, feature group 16 / 20 / 24 (generic loop + root-count skip for > 16), repeats.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_models_gpu.py -k "gbrt_root or gbrt_fused" > gpurun_out/e22_tests.log 2>&1; rc=$?; tail -1 gpurun_out/e22_tests.log; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
for kg in 16 20 24; do
  DML_TIER_KG_LARGE_REG=$kg timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/e22_c6.log 2>&1 || exit 1
  echo "[kg=$kg] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/e22_c6.log)"
  DML_GB_ROOT_CACHE=0 DML_TIER_KG_LARGE_REG=$kg timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/e22_c6.log 2>&1 || exit 1
  echo "[kg=$kg nocache] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/e22_c6.log)"
done
done
