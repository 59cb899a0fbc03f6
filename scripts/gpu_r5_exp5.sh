# Round-5 batch 5: LR skips column tiles of stopped fits (C-ordered column layout).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $PYT -m gpu tests/test_models_gpu.py tests/test_lr_device_solver.py tests/test_lr_config4_fidelity.py -k "lr or logistic or Logistic" > gpurun_out/e9_tests.log 2>&1; rc=$?; tail -2 gpurun_out/e9_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config lr --steps 3 --warmup 1 > gpurun_out/e9_lrbench.log 2>&1 && tail -1 gpurun_out/e9_lrbench.log | cut -c1-220 && grep phases gpurun_out/e9_lrbench.log | cut -c1-300 && \
DML_LR_SKIP_DONE=0 timeout -k 10 400 python -u bench.py --config lr --steps 3 --warmup 1 > gpurun_out/e9_lrbench_noskip.log 2>&1 && tail -1 gpurun_out/e9_lrbench_noskip.log | cut -c1-220
L=cs230_distributed_machine_learning_amd/lib
for v in cur epi0 pass0 pass1; do
  if [ $v = cur ]; then lib=$L/libdml_hip.so; else lib=$L/libdml_hip_$v.so; fi
  DML_HIP_LIB=$lib timeout -k 10 200 python -u scripts/lr_kernel_bench.py 10000000 1000 2560 > gpurun_out/e9_lrk_$v.log 2>&1 || exit 1
  echo "$v: $(tail -1 gpurun_out/e9_lrk_$v.log)"
done
