# Round-5 batch 22: forest runtime knobs at block_max 65536 (sweep build, min of 2 builds each).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for kv in "wave_max=384,512,640" "sub_small=24,32" "slack_wave=0,1,2" "kg_large=10,16" "block_max=65536,81920"; do
  timeout -k 10 400 python -u scripts/sweep_tiers.py $kv > gpurun_out/e30_sweep.log 2>&1 || exit 1
  grep build gpurun_out/e30_sweep.log | cut -c1-60
done
