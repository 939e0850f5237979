#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python tools/host_table_ab.py > $O/log.txt 2>&1; rc=$?
tail -5 $O/log.txt
exit $rc
