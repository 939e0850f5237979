set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_tables.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g22.log 2>&1; rc=$?; grep -E "^E  |^FAILED|passed|failed" gpurun_out/pytest_g22.log | tail -6; [ $rc = 0 ] || exit 1
timeout -k 10 400 python tools/ab_inproc.py --rounds 4 --steps 3 ov50:KS_SPLIT_FRAC=0.5 no50:KS_SPLIT_FRAC=0.5,KS_NO_P0_OVERLAP=1 ov75:KS_SPLIT_FRAC=0.75 ov90:KS_SPLIT_FRAC=0.9 ov96:KS_SPLIT_FRAC=0.96 --out gpurun_out/ab_g22.json
