set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_g5.log 2>&1 || { echo "pytest failed"; tail -50 gpurun_out/pytest_g5.log; exit 1; }
tail -2 gpurun_out/pytest_g5.log
timeout -k 10 300 python bench.py --steps 5 --out gpurun_out/b5_summ.json > gpurun_out/b5_summ.log 2>&1 || { tail -30 gpurun_out/b5_summ.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b5_summ.json')); print('summ', d['value'], d['ms_per_step'], d['phase_ms'], d['parity_sample'], d['replayed_chunks'])"
KS_NO_P1_SUMMARY=1 timeout -k 10 300 python bench.py --steps 5 --no-cpu --out gpurun_out/b5_store.json > gpurun_out/b5_store.log 2>&1 || { tail -30 gpurun_out/b5_store.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b5_store.json')); print('store', d['value'], d['ms_per_step'], d['phase_ms'], d['replayed_chunks'])"
