# LR MFMA objective: correctness of every kernel generation + A/B timings at config-4 scale.
#   gpurun -- bash scripts/gpu_lr_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $PYT -m gpu tests/test_models_gpu.py -k "lr_mfma" tests/test_lr_config4_fidelity.py > gpurun_out/lrab_tests.log 2>&1; rc=$?; tail -2 gpurun_out/lrab_tests.log; [ $rc = 0 ] || exit $rc
L=cs230_distributed_machine_learning_amd/lib
DML_LR_V3=1 timeout -k 10 200 python -u scripts/lr_kernel_bench.py 10000000 1000 2560 > gpurun_out/lrab_v3.log 2>&1 && tail -1 gpurun_out/lrab_v3.log && \
DML_LR_V3=0 timeout -k 10 200 python -u scripts/lr_kernel_bench.py 10000000 1000 2560 > gpurun_out/lrab_v2sf.log 2>&1 && tail -1 gpurun_out/lrab_v2sf.log && \
DML_LR_V3=0 DML_HIP_LIB=$L/libdml_hip_nosf.so timeout -k 10 200 python -u scripts/lr_kernel_bench.py 10000000 1000 2560 > gpurun_out/lrab_v2.log 2>&1 && tail -1 gpurun_out/lrab_v2.log && \
timeout -k 10 400 python -u bench.py --config lr --steps 2 --warmup 1 > gpurun_out/lrab_bench.log 2>&1 && tail -1 gpurun_out/lrab_bench.log | cut -c1-400 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/lrab_pmc -o p -- python3 scripts/lr_kernel_bench.py 10000000 1000 2560 > gpurun_out/lrab_pmc.log 2>&1 && echo PMC_OK
