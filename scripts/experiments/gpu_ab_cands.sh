# A/B: candidates batched per rank-step (forest batch size) on the headline metric.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in 4 8 16; do
  DML_TRACE_SYNC=0 timeout -k 10 400 python bench.py --steps 2 --warmup 1 --cands-per-rank $c > gpurun_out/cands$c.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/cands$c.log | tr '\n' ' '; echo " cands=$c"
  grep phases gpurun_out/cands$c.log | cut -c1-400
done
