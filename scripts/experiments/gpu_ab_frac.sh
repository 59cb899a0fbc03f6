set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for f in 0.55 0.8; do
  DML_HBM_FRACTION=$f timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cands-per-rank 16 > gpurun_out/fr_$f.log 2>&1 || exit 1
  echo "frac=$f $(grep -o '"value": [0-9.]*' gpurun_out/fr_$f.log) $(grep -o '"forest_batch": {"count": [0-9]*, "seconds": [0-9.]*' gpurun_out/fr_$f.log) $(grep -o '"forest_alloc": {"count": [0-9]*, "seconds": [0-9.]*' gpurun_out/fr_$f.log) $(grep -o '"forest_build": {"count": [0-9]*, "seconds": [0-9.]*' gpurun_out/fr_$f.log)"
done
