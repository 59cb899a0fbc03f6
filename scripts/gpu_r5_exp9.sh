# Round-5 batch 9: GBRT root-count cache: tests, config 6 A/B (cache off / on).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_models_gpu.py -k "gbrt" > gpurun_out/e13_tests.log 2>&1; rc=$?; tail -2 gpurun_out/e13_tests.log; [ $rc = 0 ] || exit $rc
for v in 0 1 0 1; do
  DML_GB_ROOT_CACHE=$v timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/e13_c6_$v.log 2>&1 || exit 1
  echo "cache=$v $(grep cv_fits_per_s gpurun_out/e13_c6_$v.log | cut -c1-110)"
done
