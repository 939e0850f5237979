set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g14.log 2>&1; grep -E "^E  |^FAILED|passed|failed" gpurun_out/pytest_g14.log | tail -8
for v in new old new old; do
  if [ $v = old ]; then export KS_SERIAL_ASCAN=1 KS_FIX_SERIAL=1; else unset KS_SERIAL_ASCAN KS_FIX_SERIAL; fi
  timeout -k 10 300 python bench.py --steps 5 --no-cpu --out gpurun_out/b14_$v.json > gpurun_out/b14_$v.log 2>&1 || { tail -30 gpurun_out/b14_$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b14_$v.json')); print('$v', d['value'], d['ms_per_step'], d['phase_ms'])"
done
