# A/B: forest builder variants (eval_feature inline / waves-per-EU) on the bench-like build + LR tests
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_forest_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abe_pytest.log 2>&1 && echo PYTEST_OK && \
for v in v0_noinline v1_inline v2_inline_wpe3 v3_noinline_wpe3; do DML_HIP_LIB=$PWD/variants/$v.so timeout -k 10 200 python scripts/sweep_tiers.py > gpurun_out/abe_$v.log 2>&1 || exit 1; echo "$v $(grep -o 'build [0-9.]*s' gpurun_out/abe_$v.log)"; done && \
timeout -k 10 300 python scripts/lr_objective_bench.py --rows 2000000 --features 1000 --fits 512 > gpurun_out/abe_obj.log 2>&1 && tail -1 gpurun_out/abe_obj.log
