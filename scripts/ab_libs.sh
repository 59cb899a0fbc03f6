# A/B of kernel-library variants on the bench-like forest build (scripts/sweep_tiers.py):
#   VARIANTS="base cur x2_gather" [TESTS=1] [SERIAL=1] gpurun -- bash scripts/ab_libs.sh
# "cur" = lib/libdml_hip.so, any other name = lib/libdml_hip_<name>.so (build.py --variant)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=cs230_distributed_machine_learning_amd/lib
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q tests/test_forest_gpu.py --timeout 240 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -5 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for v in ${VARIANTS}; do
  if [ "$v" = cur ]; then lib=$L/libdml_hip.so; else lib=$L/libdml_hip_$v.so; fi
  DML_HIP_LIB=$lib timeout -k 10 300 python -u scripts/sweep_tiers.py > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo "$v: $(grep build gpurun_out/ab_$v.log | tail -1 | cut -c1-60)"
done
if [ -n "$SERIAL" ]; then
  DML_SERIAL_TIERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_serial -o s -- python3 scripts/sweep_tiers.py > gpurun_out/ab_serial.log 2>&1 && echo SERIAL_OK
fi
