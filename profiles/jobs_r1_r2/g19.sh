set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() { # tag env...
  local t=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 5 --no-cpu --out gpurun_out/g19_$t.json > gpurun_out/g19_$t.log 2>&1 || { tail -20 gpurun_out/g19_$t.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/g19_$t.json')); s=d['setup_ms']; print('$t', d['value'], d['phase_ms']['scan'], s['count_ms'], s['table_first_call'])"
}
run c1 X=1 && run p1 KS_NO_CONTIG_EXT=1 && run c2 X=1 && run p2 KS_NO_CONTIG_EXT=1 && run c3 X=1 && run p3 KS_NO_CONTIG_EXT=1 && run c4 X=1 && run p4 KS_NO_CONTIG_EXT=1
