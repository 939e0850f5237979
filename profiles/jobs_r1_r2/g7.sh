set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_g7.log 2>&1; grep -E "^E  .*visits|passed|failed" gpurun_out/pytest_g7.log | tail -8
tail -1 gpurun_out/pytest_g7.log
KS_DEBUG_CARRY=1 timeout -k 10 300 python bench.py --steps 2 --no-cpu --out gpurun_out/b7_dbg.json > gpurun_out/b7_dbg.log 2>&1 || { tail -30 gpurun_out/b7_dbg.log; exit 1; }
grep -E "p1summ" gpurun_out/b7_dbg.log | tail -1
tools/ab_bench.sh g7 "--steps 5 --no-cpu" base gsumm4 base gsumm4 || exit 1
