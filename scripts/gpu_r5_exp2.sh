# Round-5 batch 2: LR bench phase breakdown + kernel stats; block-tier register variants.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=cs230_distributed_machine_learning_amd/lib
DML_TRACE_SYNC=1 timeout -k 10 400 python -u bench.py --config lr --steps 1 --warmup 1 > gpurun_out/e4_lr_phases.log 2>&1 && grep phases gpurun_out/e4_lr_phases.log | cut -c1-900 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/e4_lrprof -o p -- python3 bench.py --config lr --steps 1 --warmup 1 > gpurun_out/e4_lrprof.log 2>&1 && rm -f gpurun_out/e4_lrprof/p_kernel_trace.csv && echo LRPROF_OK && \
timeout -k 10 300 python -u scripts/sweep_tiers.py > gpurun_out/e4_cur.log 2>&1 && echo "cur: $(grep build gpurun_out/e4_cur.log)" && \
DML_HIP_LIB=$L/libdml_hip_bso.so timeout -k 10 300 python -u scripts/sweep_tiers.py > gpurun_out/e4_bso.log 2>&1 && echo "bso: $(grep build gpurun_out/e4_bso.log)" && \
DML_HIP_LIB=$L/libdml_hip_bso4.so timeout -k 10 300 python -u scripts/sweep_tiers.py > gpurun_out/e4_bso4.log 2>&1 && echo "bso4: $(grep build gpurun_out/e4_bso4.log)"
