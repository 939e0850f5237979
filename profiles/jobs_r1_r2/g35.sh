set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_g35.log 2>&1; rc=$?; tail -2 gpurun_out/smoke_g35.log; [ $rc = 0 ] || exit 1
timeout -k 10 400 python bench.py --out gpurun_out/bench_g35.json > gpurun_out/bench_g35.log 2>&1 || { tail -20 gpurun_out/bench_g35.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_g35.json')); print(d['value'], d['ms_per_step'], d['phase_ms'], d['parity_sample'], d['roofline'].get('frac'), d['roofline'].get('traffic'), d['end_to_end'], d['setup_ms']['count_ms'])"
timeout -k 10 400 python bench.py --score rank --out gpurun_out/rank_g35.json > gpurun_out/rank_g35.log 2>&1 || { tail -20 gpurun_out/rank_g35.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/rank_g35.json')); print('rank', d['value'], d['ms_per_step'], d['phase_ms'], d['parity_sample'], d['end_to_end'])"
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt35 -o kt --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu --out $R/gpurun_out/kt35_bench.json > $R/gpurun_out/kt35.log 2>&1; echo rc=$?
