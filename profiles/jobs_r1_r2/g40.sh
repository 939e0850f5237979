set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_tables.py tests/test_gpu_dual.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g40.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g40.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g40.log | head -5; [ $rc = 0 ] || exit 1
bash tools/ab_bench.sh g40 "--steps 5 --no-cpu" base viamap base viamap base viamap
