#!/bin/bash
# In-process A/B of table forms (one table per variant, all resident): wide 128-B lines, 64-B lines.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python tools/ab_inproc.py --table-per-variant --rounds 4 --steps 3 wide: l64:KS_NO_WIDE_LINES=1 "$@" > $O/ab.txt 2>&1 || { tail -30 $O/ab.txt; exit 1; }
tail -12 $O/ab.txt
