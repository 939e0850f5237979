#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
V="base: g8:KS_LANE_G8=1 hw:KS_HEADS_WIDE=1 both:KS_LANE_G8=1,KS_HEADS_WIDE=1"
timeout -k 10 500 python -u tools/ab_inproc.py --score rank --rounds 3 --steps 2 $V > $O/ab_rank.txt 2>&1 || { tail -20 $O/ab_rank.txt; exit 1; }
tail -5 $O/ab_rank.txt
