set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ingest.py tests/test_gpu_tables.py tests/test_gpu_configs.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_g16.log 2>&1; rc=$?; grep -E "^E  |^FAILED|passed|failed" gpurun_out/pytest_g16.log | tail -6; [ $rc = 0 ] || exit 1
for v in base prev base prev; do
  if [ $v = base ]; then L=kmer_spans_amd/libkmerspans.so; else L=kmer_spans_amd/libkmerspans_$v.so; fi
  KS_LIB_PATH=$PWD/$L timeout -k 10 300 python bench.py --steps 5 --no-cpu --out gpurun_out/g16_$v.json > gpurun_out/g16_$v.log 2>&1 || { tail -20 gpurun_out/g16_$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/g16_$v.json')); print('$v', d['value'], d['setup_ms']['count_ms'] if 'setup_ms' in d else d.get('setup'), d['end_to_end'])"
done
