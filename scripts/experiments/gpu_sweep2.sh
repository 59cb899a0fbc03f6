set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
S=scripts/sweep_tiers.py
timeout -k 10 400 python -u $S block_max=8192,16384,32768 chunk=8192,16384,32768 > gpurun_out/sw_a.log 2>&1 && echo A_OK && \
timeout -k 10 300 python -u $S wave_max=128,192,256,384 sub_max=32,64 > gpurun_out/sw_b.log 2>&1 && echo B_OK && \
for v in rpt2 wpe2 kgw2; do DML_HIP_LIB=variants/$v.so timeout -k 10 120 python -u $S > gpurun_out/sw_v_$v.log 2>&1 || exit 1; done && echo V_OK
