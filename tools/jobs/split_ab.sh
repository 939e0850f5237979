#!/bin/bash
# In-process A/B of the split fraction of the two concurrent halves.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 500 python tools/ab_inproc.py --rounds 4 --steps 3 f70: f65:KS_SPLIT_FRAC=0.65 f60:KS_SPLIT_FRAC=0.6 f55:KS_SPLIT_FRAC=0.55 f50:KS_SPLIT_FRAC=0.5 "$@" > $O/ab.txt 2>&1 || { tail -30 $O/ab.txt; exit 1; }
cat $O/ab.txt | tail -20
