# Round-5 experiment batch: LR v3 epilogue check + forest tier/occupancy A/B.
#   gpurun -- bash scripts/gpu_r5_exp.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
L=cs230_distributed_machine_learning_amd/lib
timeout -k 10 400 $PYT -m gpu tests/test_models_gpu.py -k "lr_mfma" tests/test_lr_config4_fidelity.py > gpurun_out/e3_tests.log 2>&1; rc=$?; tail -2 gpurun_out/e3_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u scripts/lr_kernel_bench.py 10000000 1000 2560 > gpurun_out/e3_lrk.log 2>&1 && tail -1 gpurun_out/e3_lrk.log && \
timeout -k 10 400 python -u bench.py --config lr --steps 2 --warmup 1 > gpurun_out/e3_lrbench.log 2>&1 && tail -1 gpurun_out/e3_lrbench.log | cut -c1-200 && \
timeout -k 10 300 python -u scripts/sweep_tiers.py kg_block=10,12,16 > gpurun_out/e3_kgb.log 2>&1 && cat gpurun_out/e3_kgb.log | grep build && \
DML_HIP_LIB=$L/libdml_hip_wv3.so timeout -k 10 300 python -u scripts/sweep_tiers.py > gpurun_out/e3_wv3.log 2>&1 && echo "wv3: $(grep build gpurun_out/e3_wv3.log)" && \
DML_HIP_LIB=$L/libdml_hip_wb4.so timeout -k 10 300 python -u scripts/sweep_tiers.py > gpurun_out/e3_wb4.log 2>&1 && echo "wb4: $(grep build gpurun_out/e3_wb4.log)"
