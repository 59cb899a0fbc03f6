# Round-5: kernel stats of GBRT config 6 at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/e27_prof -o p -- python3 scripts/bench_configs.py --configs 6 > gpurun_out/e27_prof.log 2>&1 && \
f=$(find gpurun_out/e27_prof -name "*kernel_stats.csv" | head -1) && cp $f gpurun_out/e27_c6_kernel_stats.csv && head -14 gpurun_out/e27_c6_kernel_stats.csv | cut -c1-140 && \
python scripts/timeline.py gpurun_out/e27_prof k_gb_grad | head -3; rc=$?
find gpurun_out/e27_prof -name "*.csv" -size +20M -delete; exit $rc
