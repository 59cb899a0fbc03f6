# A/B: bigger forest batches (HBM fraction) x candidates per rank-step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, cands, frac
  DML_HBM_FRACTION=$3 timeout -k 10 500 python bench.py --steps 2 --warmup 1 --cands-per-rank $2 > gpurun_out/$1.log 2>&1 || return 1
  echo "$1 $(grep -o '"value": [0-9.]*' gpurun_out/$1.log) batches=$(grep -o '"forest_batch": {"count": [0-9]*' gpurun_out/$1.log)"
}
run c16f55 16 0.55 && run c16f85 16 0.85 && run c32f85 32 0.85
