#!/bin/bash
# The weighted-rank bench lines (config 3 k = 13, config 4 k = 15) with their
# parity legs.  Usage: tools/gpu_rank_lines.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
run() { tag=$1; shift; timeout -k 10 600 python bench.py --out $O/cfg_$tag.json "$@" > $O/cfg_$tag.log 2>&1 || { echo "FAILED $tag"; tail -20 $O/cfg_$tag.log; exit 1; }; python3 -c "import json;b=json.load(open('$O/cfg_$tag.json'));print('$tag', b['value'], b['ms_per_step'], b.get('parity_sample'), b['phase_ms'].get('total'))"; }
run cfg3_rank_k13 --score rank --k 13 --steps 3 --warmup 1 --no-rank --no-host-path --no-visits
run cfg4_rank_k15 --score rank --k 15 --steps 3 --warmup 1 --no-rank --no-host-path --no-visits
