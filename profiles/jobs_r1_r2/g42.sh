set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g42.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g42.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g42.log | head -5; [ $rc = 0 ] || exit 1
bash tools/ab_bench.sh g42 "--steps 5 --no-cpu" base prev base prev base prev
