set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g30.log 2>&1; rc=$?; grep -E "^E  |^FAILED|passed|failed" gpurun_out/pytest_g30.log | tail -8; [ $rc = 0 ] || exit 1
timeout -k 10 400 python tools/ab_inproc.py --rounds 3 --steps 3 batch: nobatch:KS_NO_TILE_BATCH=1 --out gpurun_out/ab_g30.json || exit 1
KS_DEBUG_CARRY=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --out gpurun_out/g30.json > gpurun_out/g30.log 2>&1; grep "\[carry\]" gpurun_out/g30.log | head -5
