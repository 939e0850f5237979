#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python -u tools/ab_inproc.py --rounds 4 --steps 3 base: nopf:KS_PREDICT_NOPF=1 > $O/ab_genome.txt 2>&1 || { tail -20 $O/ab_genome.txt; exit 1; }
tail -3 $O/ab_genome.txt
timeout -k 10 400 python -u tools/ab_inproc.py --rounds 4 --steps 3 --shard-of 8 base: nopf:KS_PREDICT_NOPF=1 > $O/ab_shard8.txt 2>&1 || { tail -20 $O/ab_shard8.txt; exit 1; }
tail -3 $O/ab_shard8.txt
