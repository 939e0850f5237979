set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_smallk.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g15.log 2>&1; grep -E "^E  |^FAILED|passed|failed" gpurun_out/pytest_g15.log | tail -6
tools/ab_bench.sh g15 "--steps 5 --no-cpu" base prev base prev || exit 1
