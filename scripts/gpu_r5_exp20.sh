# Round-5 batch 20: forest tier knob re-sweep at HEAD (sweep build, min of 2 builds each).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for kv in "wave_max=384,512,768" "block_max=16384,32768,65536" "sub_small=16,32" "kg_block=8,12,16" "chunk=8192,16384,32768" "kg_wave=2,3,4"; do
  timeout -k 10 400 python -u scripts/sweep_tiers.py $kv > gpurun_out/e28_sweep.log 2>&1 || exit 1
  grep build gpurun_out/e28_sweep.log | cut -c1-70
done
