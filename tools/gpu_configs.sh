#!/bin/bash
# Every BASELINE.json configuration that fits one GPU (and this project's own
# lines), one bench.py JSON line each, parity against the oracle included.
# Usage: tools/gpu_configs.sh TAG [PART]  (PART: a = lines 1-5, b = lines 6-9, default both)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-cfg}
P=${2:-ab}
mkdir -p $OUT
cd $R
run() { tag=$1; shift; timeout -k 10 600 python bench.py --out $OUT/cfg_$tag.json "$@" > $OUT/cfg_$tag.log 2>&1 || { echo "FAILED $tag"; tail -20 $OUT/cfg_$tag.log; exit 1; }; python3 -c "import json;b=json.load(open('$OUT/cfg_$tag.json'));print('$tag', b['value'], b['ms_per_step'], b.get('parity_sample'), (b.get('roofline') or {}).get('frac'))"; }
if [[ $P == *a* ]]; then
run cfg2_chr1_k11 --ncontigs 1 --k 11 --steps 5 --warmup 1 --no-rank --no-host-path --no-visits
run cfg3_pm1_k13 --score pm1 --k 13 --steps 5 --warmup 1 --no-rank --no-host-path --no-visits
run cfg4_log2_k15 --k 15 --steps 3 --warmup 1 --no-rank --no-host-path --no-visits
run cfg4_rank_k15 --score rank --k 15 --steps 3 --warmup 1 --no-rank --no-host-path --no-visits
run cfg3_rank_k13 --score rank --k 13 --steps 3 --warmup 1 --no-rank --no-host-path --no-visits
fi
if [[ $P == *b* ]]; then
run small_k7_pm1 --k 7 --score pm1 --steps 5 --warmup 1 --no-rank --no-host-path --no-visits
run trlr_k13 --trlr --steps 3 --warmup 1 --no-rank --no-host-path --no-visits
run shardof8 --shard-of 8 --steps 10 --warmup 2 --no-rank --no-host-path --no-visits --no-cpu
run cfg5_genomes --mode genomes --genomes-per-rank 4
fi
