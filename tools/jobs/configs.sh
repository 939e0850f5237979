#!/bin/bash
# BASELINE configuration lines on one GPU (besides the default metric line).  Usage: tools/jobs/configs.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
run() { tag=$1; shift; timeout -k 10 500 python bench.py --out $O/cfg_$tag.json "$@" > $O/cfg_$tag.log 2>&1 || { echo "FAILED $tag"; tail -20 $O/cfg_$tag.log; exit 1; }
  python -c "import json;b=json.load(open('$O/cfg_$tag.json'));print('$tag', b['value'], b['ms_per_step'], b.get('parity_sample'), b.get('parity_bp'), b['config'].get('pass1_kernel'), b['config'].get('positions_per_read'), (b.get('end_to_end') or {}).get('ms'))"; }
run cfg2_chr1_k11 --ncontigs 1 --k 11 --steps 5 --warmup 1 --no-rank --no-host-path
run cfg4_log2_k15 --k 15 --steps 3 --warmup 1 --no-rank --no-host-path --parity sample
run cfg4_rank_k15 --k 15 --score rank --steps 3 --warmup 1 --no-rank --no-host-path --parity sample
run cfg5_genomes --mode genomes --genomes-per-rank 2 --steps 1 --warmup 1
run trlr_k13 --trlr --steps 3 --warmup 1 --no-rank --no-host-path --no-visits --parity sample
run pm1_k13 --score pm1 --steps 3 --warmup 1 --no-rank --no-host-path --no-visits --parity sample
run small_k7 --k 7 --score pm1 --steps 5 --warmup 1 --no-rank --no-host-path --no-visits --parity sample
