set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ingest.py tests/test_gpu_parity.py tests/test_gpu_tables.py tests/test_gpu_smallk.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g33.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g33.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g33.log | head -5; [ $rc = 0 ] || exit 1
timeout -k 10 300 python tools/ab_count.py base: && timeout -k 10 300 python tools/ab_count.py --k 11 k11: && timeout -k 10 300 python tools/ab_count.py --k 7 k7: && timeout -k 10 300 python tools/ab_count.py --k 15 k15:
