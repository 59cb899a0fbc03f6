# Round-5 batch 6: v3 LR MFMA-pass probes, block-tier phase profile at HEAD, RF bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=cs230_distributed_machine_learning_amd/lib
for v in pass0 pass1; do
  DML_HIP_LIB=$L/libdml_hip_$v.so timeout -k 10 200 python -u scripts/lr_kernel_bench.py 10000000 1000 2560 > gpurun_out/e10_lrk_$v.log 2>&1 || exit 1
  echo "$v: $(tail -1 gpurun_out/e10_lrk_$v.log)"
done
DML_HIP_LIB=$L/libdml_hip_phase.so timeout -k 10 300 python -u scripts/phase_prof.py > gpurun_out/e10_phase.log 2>&1 && tail -3 gpurun_out/e10_phase.log && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/e10_bench.log 2>&1 && tail -1 gpurun_out/e10_bench.log | cut -c1-200
