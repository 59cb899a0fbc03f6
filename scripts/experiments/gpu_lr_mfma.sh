# MFMA LR objective: numerics tests, objective microbench, BASELINE config 4 (10M x 1000).
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -v --timeout 120 --timeout-method thread -k "mfma or lr_" > gpurun_out/lrm_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python scripts/lr_objective_bench.py --rows 2000000 --features 1000 --fits 512 > gpurun_out/lrm_obj.log 2>&1 && tail -1 gpurun_out/lrm_obj.log && \
timeout -k 10 600 python scripts/bench_configs.py --configs 4 --lr-rows 10000000 > gpurun_out/lrm_cfg4.log 2>&1 && grep cv_fits gpurun_out/lrm_cfg4.log
