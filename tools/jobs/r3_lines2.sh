#!/bin/bash
# r3: pass-1 memory patterns for a continuation-line table (tools/line_bench2.hip).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3_lines2
mkdir -p $O
cd $R
timeout -k 10 300 ./tools/line_bench2 128 > $O/line_bench2.txt 2>&1; rc=$?
cat $O/line_bench2.txt
exit $rc
