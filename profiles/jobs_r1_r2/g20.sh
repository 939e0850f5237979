set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() { # tag env...
  local t=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 5 --no-cpu --out gpurun_out/g20_$t.json > gpurun_out/g20_$t.log 2>&1 || { tail -20 gpurun_out/g20_$t.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/g20_$t.json')); print('$t', d['value'], d['ms_per_step'], d['phase_ms'], d.get('parity_sample',{}).get('ok') if isinstance(d.get('parity_sample'),dict) else d.get('parity_sample'))"
}
run f50 KS_SPLIT_FRAC=0.5 && run f65 KS_SPLIT_FRAC=0.65 && run f75 KS_SPLIT_FRAC=0.75 && run f85 KS_SPLIT_FRAC=0.85 && run f92 KS_SPLIT_FRAC=0.92 && run f50b KS_SPLIT_FRAC=0.5 && run f75b KS_SPLIT_FRAC=0.75
