set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g49.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g49.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g49.log | head -5; [ $rc = 0 ] || exit 1
KS_DEBUG_CARRY=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --out gpurun_out/g49.json > gpurun_out/g49.log 2>&1; grep "\[carry\]\|\[replay\|\[p1summ" gpurun_out/g49.log | head -6
timeout -k 10 400 python tools/ab_inproc.py --rounds 4 --steps 3 pre: nopre:KS_NO_REPLAY_PREFETCH=1 --out gpurun_out/ab_g49.json
