# A/B of the predict kernel's lock-step width (DML_PRED_U 4/8/16): kernel stats per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for u in 8 16 4; do
  DML_PRED_U=$u timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/predu$u -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/predu$u.log 2>&1 || exit 1
  python scripts/summarize_prof.py /tmp/predu$u > gpurun_out/predu${u}_stats.txt 2>&1 || exit 1
  grep -o '"value": [0-9.]*' gpurun_out/predu$u.log
done
grep -H "predict" gpurun_out/predu*_stats.txt
