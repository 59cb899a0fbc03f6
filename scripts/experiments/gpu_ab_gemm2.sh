set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "mfma or lr_" > gpurun_out/abg2_pytest.log 2>&1 && echo PYTEST_OK && \
for v in g0_base g6_regstage; do DML_HIP_LIB=$PWD/variants/$v.so timeout -k 10 120 python scripts/lr_kernel_bench.py > gpurun_out/abg2_$v.log 2>&1 || exit 1; tail -1 gpurun_out/abg2_$v.log; done && \
timeout -k 10 300 python scripts/lr_objective_bench.py --rows 2000000 --features 1000 --fits 512 > gpurun_out/abg2_obj.log 2>&1 && tail -1 gpurun_out/abg2_obj.log
