set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g61.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g61.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g61.log | head -5; [ $rc = 0 ] || exit 1
timeout -k 10 400 python tools/ab_inproc.py --rounds 4 --steps 3 hi: side:KS_TAIL_ON_SIDE=1 --out gpurun_out/ab_g61.json
