# Round-5 batch 13: LR v4 forward kernel timing (fixed harness) v4 vs v3.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 1 0; do
  DML_LR_V4=$v timeout -k 10 200 python -u scripts/lr_kernel_bench.py 10000000 1000 2560 > gpurun_out/e18_lrk_v4$v.log 2>&1 || exit 1
  echo "v4=$v $(tail -1 gpurun_out/e18_lrk_v4$v.log)"
done
