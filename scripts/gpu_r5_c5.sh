# Round-5: config 5 (mixed queue) local runner vs the cluster runner at world 1, interleaved x3.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs 5 > gpurun_out/e14_local$i.log 2>&1 || exit 1
  echo "local$i $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/e14_local$i.log)"
  DML_FORCE_PG=1 timeout -k 10 300 python -u scripts/bench_configs.py --configs 5 > gpurun_out/e14_dist$i.log 2>&1 || exit 1
  echo "dist$i $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/e14_dist$i.log)"
done
