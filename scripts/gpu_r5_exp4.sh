# Round-5 batch 4: LR epilogue vector reads + batched binary predictions; block-tier partition row keep A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
L=cs230_distributed_machine_learning_amd/lib
timeout -k 10 400 $PYT -m gpu tests/test_models_gpu.py -k "lr_mfma or logistic" > gpurun_out/e6_tests.log 2>&1; rc=$?; tail -2 gpurun_out/e6_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u scripts/lr_kernel_bench.py 10000000 1000 2560 > gpurun_out/e6_lrk.log 2>&1 && tail -1 gpurun_out/e6_lrk.log && \
timeout -k 10 400 python -u bench.py --config lr --steps 3 --warmup 1 > gpurun_out/e6_lrbench.log 2>&1 && tail -1 gpurun_out/e6_lrbench.log | cut -c1-220 && grep phases gpurun_out/e6_lrbench.log | cut -c1-400 && \
for v in cur pk1 pk2; do
  if [ $v = cur ]; then lib=$L/libdml_hip.so; else lib=$L/libdml_hip_$v.so; fi
  DML_HIP_LIB=$lib timeout -k 10 300 python -u scripts/sweep_tiers.py > gpurun_out/e6_$v.log 2>&1 || exit 1
  echo "$v: $(grep build gpurun_out/e6_$v.log | cut -c1-60)"
done && \
DML_HIP_LIB=$L/libdml_hip_pk2.so timeout -k 10 300 $PYT -m gpu tests/test_forest_gpu.py tests/test_forest_tiers.py > gpurun_out/e6_pk2tests.log 2>&1; rc=$?; tail -1 gpurun_out/e6_pk2tests.log; exit $rc
