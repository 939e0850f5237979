set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() { # tag lib env...
  local t=$1 v=$2; shift 2
  if [ $v = base ]; then L=kmer_spans_amd/libkmerspans.so; else L=kmer_spans_amd/libkmerspans_$v.so; fi
  env "$@" KS_LIB_PATH=$PWD/$L timeout -k 10 300 python bench.py --steps 5 --no-cpu --out gpurun_out/g18_$t.json > gpurun_out/g18_$t.log 2>&1 || { tail -20 gpurun_out/g18_$t.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/g18_$t.json')); s=d['setup_ms']; print('$t', d['value'], d['phase_ms']['scan'], s['count_ms'], s['table_first_call'])"
}
run b1 base X=1 && run c1 base KS_CNT_RES_C=1 && run bc1 base KS_CNT_RES_C=1 KS_CNT_RES_B=1 && run p1 prev X=1 && run b2 base X=1 && run c2 base KS_CNT_RES_C=1 && run bc2 base KS_CNT_RES_C=1 KS_CNT_RES_B=1 && run p2 prev X=1
