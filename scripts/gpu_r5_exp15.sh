# Round-5 batch 15b: GBRT config 6, regression large-tier feature group size (interleaved repeats).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for v in "DML_TIER_KG_LARGE_REG=16" "DML_TIER_KG_LARGE_REG=20" "DML_TIER_KG_LARGE_REG=25" "DML_TIER_KG_LARGE_REG=34"; do
  env $v timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/e20_c6.log 2>&1 || exit 1
  echo "[$v] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/e20_c6.log)"
done
done
