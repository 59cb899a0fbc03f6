# RCCL path on one GPU: forced world-1 nccl group test, GPU test tier, bench through the
# process group (DML_FORCE_PG=1), and a kernel trace proving RCCL kernels ran.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/rccl_test.log 2>&1; echo "rccl test rc=$?"; tail -3 gpurun_out/rccl_test.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_all.log 2>&1; echo "gpu tier rc=$?"; tail -2 gpurun_out/gpu_all.log
DML_FORCE_PG=1 MASTER_PORT=29581 timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_pg.log 2>&1 && tail -1 gpurun_out/bench_pg.log | cut -c1-160 && \
DML_FORCE_PG=1 MASTER_PORT=29582 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rccl_prof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/rccl_prof.log 2>&1 && echo PROF_OK
