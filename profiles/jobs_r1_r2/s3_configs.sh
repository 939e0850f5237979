#!/bin/bash
# Session-3: every BASELINE.json configuration that fits one GPU on the final
# build, one JSON line each (config 5 as genomes-per-rank on one GPU).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/s3cfg
mkdir -p $OUT
cd $R
run() { tag=$1; shift; timeout -k 10 400 python bench.py --out $OUT/cfg_$tag.json "$@" > $OUT/cfg_$tag.log 2>&1 || { echo "FAILED $tag"; tail -20 $OUT/cfg_$tag.log; exit 1; }; }
run metric_host --steps 5 --warmup 1 --host-path --no-cpu
run cfg2_chr1_k11 --ncontigs 1 --k 11 --steps 5 --warmup 1
run cfg3_rank_k13 --score rank --k 13 --steps 3 --warmup 1
run cfg4_log2_k15 --k 15 --steps 3 --warmup 1
run cfg5_genomes --mode genomes --genomes-per-rank 2 --no-cpu
run trlr_k13 --trlr --steps 3 --warmup 1 --no-cpu
