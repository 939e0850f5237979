#!/bin/bash
# A/B bench of library variants on one box: tools/ab_bench.sh TAG "bench args" variant...
# (variant "base" = the in-tree build, else kmer_spans_amd/libkmerspans_<v>.so)
set -o pipefail
TAG=$1; ARGS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in "$@"; do
  if [ "$v" = base ]; then L=$R/kmer_spans_amd/libkmerspans.so; else L=$R/kmer_spans_amd/libkmerspans_$v.so; fi
  KS_LIB_PATH=$L timeout -k 10 300 python bench.py $ARGS --out gpurun_out/ab_${TAG}_$v.json > gpurun_out/ab_${TAG}_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/ab_${TAG}_$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_$v.json')); print('$v', d['value'], d['ms_per_step'], d['phase_ms'], d.get('parity_sample'), d['regions'])"
done
