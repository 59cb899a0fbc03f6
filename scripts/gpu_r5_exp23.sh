# Round-5 batch 23: forest compile-time knob variants at HEAD (sweep build, min of 2 builds), repeated.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=cs230_distributed_machine_learning_amd/lib
for rep in 1 2; do
for v in cur wpe3 wpe5 pf10 gpf0 win2 lnf0; do
  if [ $v = cur ]; then lib=$L/libdml_hip.so; else lib=$L/libdml_hip_$v.so; fi
  DML_HIP_LIB=$lib timeout -k 10 300 python -u scripts/sweep_tiers.py > gpurun_out/e31_$v.log 2>&1 || exit 1
  echo "$v: $(grep build gpurun_out/e31_$v.log | cut -c1-40)"
done
done
