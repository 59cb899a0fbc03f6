# Round-5 batch 11: fused percentile-loss GBRT stages: tests, config-6 huber fused vs torch, kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_models_gpu.py -k "gbrt" > gpurun_out/e16_tests.log 2>&1; rc=$?; tail -2 gpurun_out/e16_tests.log; [ $rc = 0 ] || exit $rc
for v in 1 0; do
  DML_GB_FUSED=$v timeout -k 10 400 python -u scripts/bench_configs.py --configs 6 --gb-loss huber > gpurun_out/e16_huber_f$v.log 2>&1 || exit 1
  echo "fused=$v $(grep cv_fits_per_s gpurun_out/e16_huber_f$v.log | cut -c1-200)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/e16_prof -o p -- python3 scripts/bench_configs.py --configs 6 --gb-loss huber > gpurun_out/e16_prof.log 2>&1 && \
f=$(find gpurun_out/e16_prof -name "*kernel_stats.csv" | head -1) && cp $f gpurun_out/e16_huber_kernel_stats.csv && head -25 gpurun_out/e16_huber_kernel_stats.csv | cut -c1-150; rc=$?
find gpurun_out/e16_prof -name "*.csv" -size +20M -delete; exit $rc
