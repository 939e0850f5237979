set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g23.log 2>&1; rc=$?; grep -E "^E  |^FAILED|passed|failed" gpurun_out/pytest_g23.log | tail -6; [ $rc = 0 ] || exit 1
timeout -k 10 500 python tools/ab_inproc.py --rounds 4 --steps 3 ser50:KS_SPLIT_FRAC=0.5,KS_P1_SERIAL_HALVES=1 ser96:KS_SPLIT_FRAC=0.96,KS_P1_SERIAL_HALVES=1 con50:KS_SPLIT_FRAC=0.5 con65:KS_SPLIT_FRAC=0.65 con80:KS_SPLIT_FRAC=0.8 con90:KS_SPLIT_FRAC=0.9 --out gpurun_out/ab_g23.json
