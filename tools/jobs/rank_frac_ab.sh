#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
V="f70: f60:KS_SPLIT_FRAC=0.6 f80:KS_SPLIT_FRAC=0.8 f90:KS_SPLIT_FRAC=0.9 one:KS_NO_F64_SPLIT=1"
timeout -k 10 500 python -u tools/ab_inproc.py --score rank --rounds 3 --steps 2 $V > $O/ab_rank_frac.txt 2>&1 || { tail -20 $O/ab_rank_frac.txt; exit 1; }
tail -6 $O/ab_rank_frac.txt
