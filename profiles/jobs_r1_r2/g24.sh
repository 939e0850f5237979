set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g24.log 2>&1; rc=$?; grep -E "^E  |^FAILED|passed|failed" gpurun_out/pytest_g24.log | tail -6; [ $rc = 0 ] || exit 1
timeout -k 10 500 python tools/ab_inproc.py --rounds 3 --steps 3 ser50:KS_SPLIT_FRAC=0.5,KS_P1_SERIAL_HALVES=1 c60:KS_SPLIT_FRAC=0.6 c65: c70:KS_SPLIT_FRAC=0.7 nosplit:KS_NO_SPLIT=1 --out gpurun_out/ab_g24.json
timeout -k 10 400 python bench.py --out gpurun_out/bench_g24.json > gpurun_out/bench_g24.log 2>&1 || { tail -20 gpurun_out/bench_g24.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_g24.json')); print(d['value'], d['ms_per_step'], d['phase_ms'], d['parity_sample'], d['cpu_baseline'])"
