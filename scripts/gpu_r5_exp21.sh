# Round-5 batch 21: forest block_max re-sweep (repeats), then the headline bench at the best value.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 400 python -u scripts/sweep_tiers.py block_max=32768,49152,65536,98304,131072 > gpurun_out/e29_sweep.log 2>&1 || exit 1
  grep build gpurun_out/e29_sweep.log | cut -c1-60
done
for bm in 32768 65536 32768 65536; do
  DML_TIER_BLOCK_MAX=$bm timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/e29_bench.log 2>&1 || exit 1
  echo "bench block_max=$bm $(tail -1 gpurun_out/e29_bench.log | cut -c90-130)"
done
