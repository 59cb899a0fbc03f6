# Round-5 batch 19: GBRT config 6 with 1 / 2 / 3 / 4 build lanes (repeats).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for L in 2 3 4 1; do
  DML_GB_LANES=$L timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/e26_c6.log 2>&1 || exit 1
  echo "[lanes=$L] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/e26_c6.log)"
done
done
