set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for t in 1 2 3 4 5; do
  KS_DEBUG_ALLOC=1 timeout -k 10 300 python bench.py --steps 5 --no-cpu --out gpurun_out/g21_$t.json > gpurun_out/g21_$t.log 2>&1 || { tail -20 gpurun_out/g21_$t.log; exit 1; }
  grep "ext alloc" gpurun_out/g21_$t.log | head -3
  python3 -c "import json; d=json.load(open('gpurun_out/g21_$t.json')); print('$t', d['value'], d['phase_ms']['scan'], d['setup_ms']['table_first_call'])"
done
