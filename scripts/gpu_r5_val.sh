# Round-5 validation at HEAD: forest/model GPU tests, headline bench, level spans of the sweep build.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r5v}
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 800 $PYT -m gpu tests/test_forest_gpu.py tests/test_forest_tiers.py tests/test_models_gpu.py tests/test_binned_only.py > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1 && tail -1 gpurun_out/${T}_bench.log | cut -c1-200 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/${T}_lv -o lv -- python3 scripts/sweep_tiers.py > gpurun_out/${T}_lv.log 2>&1 && \
python scripts/level_spans.py $(find gpurun_out/${T}_lv -name "*.db" | head -1) > gpurun_out/${T}_levels.txt && head -20 gpurun_out/${T}_levels.txt && find gpurun_out/${T}_lv -name "*.db" -delete
