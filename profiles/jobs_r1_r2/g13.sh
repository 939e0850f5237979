set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g13.log 2>&1; grep -E "^E  |^FAILED|passed|failed" gpurun_out/pytest_g13.log | tail -8
timeout -k 10 300 python bench.py --steps 5 --out gpurun_out/b13_split.json > gpurun_out/b13_split.log 2>&1 || { tail -30 gpurun_out/b13_split.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b13_split.json')); print('split', d['value'], d['ms_per_step'], d['phase_ms'], d['parity_sample'], d['table_equal_host'])"
KS_NO_SPLIT=1 timeout -k 10 300 python bench.py --steps 5 --no-cpu --out gpurun_out/b13_nosplit.json > gpurun_out/b13_nosplit.log 2>&1 || { tail -30 gpurun_out/b13_nosplit.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b13_nosplit.json')); print('nosplit', d['value'], d['ms_per_step'], d['phase_ms'])"
timeout -k 10 300 python bench.py --steps 5 --no-cpu --out gpurun_out/b13_split2.json > gpurun_out/b13_split2.log 2>&1 || { tail -30 gpurun_out/b13_split2.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b13_split2.json')); print('split', d['value'], d['ms_per_step'], d['phase_ms'])"
