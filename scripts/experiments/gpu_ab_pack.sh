# Same-box A/B of packed leaf probabilities in predict (DML_PACK_LEAVES 0/1), twice each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1 0 1; do
  DML_PACK_LEAVES=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk$v -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/pkab$v.log 2>&1 || exit 1
  python scripts/summarize_prof.py /tmp/pk$v > gpurun_out/pkab${v}_stats.txt 2>&1 || exit 1
  rm -rf /tmp/pk$v
  echo "pack=$v $(grep predict gpurun_out/pkab${v}_stats.txt | cut -c1-130)"
done
