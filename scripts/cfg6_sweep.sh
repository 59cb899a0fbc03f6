# config-6 (GBRT) tier sweep: one bench_configs run per setting (GPU box).  Settings are
# DML_TIER_<FIELD>=<int> overrides of ops/forest_ops.py ForestTiers and forest.hip knobs.
set -o pipefail
for cfg in "X=0" "X=0" "X=0"; do
  env $cfg timeout -k 10 200 python -u scripts/bench_configs.py --configs 6 > gpurun_out/sw.log 2>&1 || exit 1
  echo "$cfg $(grep -o '"cv_fits_per_s": [0-9.]*' gpurun_out/sw.log)" | tee -a gpurun_out/cfg6_sweep.txt
done
