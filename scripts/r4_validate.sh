# round-4 GPU check: forest/model GPU tests, headline bench x2, a wave_max variant, config 6 x3
set -o pipefail
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_forest_gpu.py tests/test_models_gpu.py tests/test_reg_fixed_point.py > gpurun_out/t_w.log 2>&1 || exit 1
tail -1 gpurun_out/t_w.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bw$i.log 2>&1 || exit 1
  tail -1 gpurun_out/bw$i.log | cut -c1-150
done
DML_TIER_WAVE_MAX=256 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bw256.log 2>&1 || exit 1
echo "wave_max 256: $(tail -1 gpurun_out/bw256.log | cut -c90-150)"
bash scripts/cfg6_sweep.sh
