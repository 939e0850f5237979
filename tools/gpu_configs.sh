#!/bin/bash
# Every BASELINE.json configuration that fits one GPU, one JSON line each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
cd $R
run() { tag=$1; shift; timeout -k 10 600 python bench.py --out $OUT/cfg_$tag.json "$@" > $OUT/cfg_$tag.log 2>&1 || { echo "FAILED $tag"; tail -20 $OUT/cfg_$tag.log; exit 1; }; cat $OUT/cfg_$tag.json; }
run metric --steps 5 --warmup 1 --host-path
run cfg2_chr1_k11 --ncontigs 1 --k 11 --steps 5 --warmup 1
run cfg3_rank_k13 --score rank --k 13 --steps 3 --warmup 1
run cfg3_pm1_k13 --score pm1 --k 13 --steps 3 --warmup 1
run cfg4_log2_k15 --k 15 --steps 3 --warmup 1
run noexpand_k13 --no-expand --steps 3 --warmup 1 --no-cpu
