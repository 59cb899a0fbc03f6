# Round-5: kernel stats of the headline bench at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/e25_prof -o p -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/e25_prof.log 2>&1 && \
f=$(find gpurun_out/e25_prof -name "*kernel_stats.csv" | head -1) && cp $f gpurun_out/e25_bench_kernel_stats.csv && head -16 gpurun_out/e25_bench_kernel_stats.csv | cut -c1-140; rc=$?
find gpurun_out/e25_prof -name "*.csv" -size +20M -delete; exit $rc
