# Round-5 batch 8: GBRT config 6: tests, lanes A/B, kernel trace of the 2-lane run -> busy union + idle gaps.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_models_gpu.py -k "gbrt" > gpurun_out/e12_tests.log 2>&1; rc=$?; tail -2 gpurun_out/e12_tests.log; [ $rc = 0 ] || exit $rc
for L in 1 2 1 2; do
  DML_GB_LANES=$L timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/e12_c6_l$L.log 2>&1 || exit 1
  echo "lanes=$L $(grep cv_fits_per_s gpurun_out/e12_c6_l$L.log | cut -c1-100)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/e12_tr -o t -- python3 scripts/bench_configs.py --configs 6 > gpurun_out/e12_tr.log 2>&1 && \
python scripts/timeline.py gpurun_out/e12_tr 0.3 > gpurun_out/e12_busy.txt && head -14 gpurun_out/e12_busy.txt && \
python scripts/gaps.py gpurun_out/e12_tr 20 0.3 > gpurun_out/e12_gaps.txt && head -20 gpurun_out/e12_gaps.txt; rc=$?
find gpurun_out/e12_tr -name "*.csv" -size +20M -delete; exit $rc
