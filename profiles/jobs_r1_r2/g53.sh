set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g53.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g53.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g53.log | head -5; [ $rc = 0 ] || exit 1
timeout -k 10 500 python tools/ab_inproc.py --score rank --rounds 3 --steps 2 pre: nopre:KS_NO_REPLAY_PREFETCH=1 --out gpurun_out/ab_g53.json
