set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dual.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_g34a.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_g34a.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g34a.log | head -8; [ $rc = 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g34.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g34.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g34.log | head -5; [ $rc = 0 ] || exit 1
timeout -k 10 400 python tools/ab_inproc.py --rounds 3 --steps 3 dual: one:KS_NO_DUAL=1 dual_nosplit:KS_NO_SPLIT=1 --out gpurun_out/ab_g34.json
