set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -v --timeout 120 --timeout-method thread -k "mfma or lr_" > gpurun_out/lrm2_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python scripts/lr_objective_bench.py --rows 2000000 --features 1000 --fits 512 > gpurun_out/lrm2_obj.log 2>&1 && tail -1 gpurun_out/lrm2_obj.log && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lrobj2 -o o -- python3 scripts/lr_objective_bench.py --rows 2000000 --features 1000 --fits 512 > gpurun_out/prof_lrobj2.log 2>&1 && echo PROF_OK
