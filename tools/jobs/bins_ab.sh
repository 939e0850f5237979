#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_count.py --rounds 3 --steps 2 --k 13 old:KS_SCATTER_STAGE=0 base: > $O/ab_k13.txt 2>&1 || { tail -20 $O/ab_k13.txt; exit 1; }
tail -4 $O/ab_k13.txt
for K in 11 12 14; do
timeout -k 10 200 python -u tools/ab_count.py --rounds 1 --steps 1 --k $K --scale 0.1 old:KS_SCATTER_STAGE=0 base: > $O/ab_k$K.txt 2>&1 || { tail -20 $O/ab_k$K.txt; exit 1; }
tail -4 $O/ab_k$K.txt
done
