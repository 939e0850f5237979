#!/bin/bash
# Weighted rank (config 3) in process: FP64 line table vs the FP64 (k+3)-mer table.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python tools/ab_inproc.py --score rank --table-per-variant --rounds 3 --steps 3 lines: ext:KS_NO_LINES=1 "$@" > $O/ab.txt 2>&1 || { tail -30 $O/ab.txt; exit 1; }
tail -8 $O/ab.txt
