#!/bin/bash
# Kernel trace of the weighted-rank step (config 3) in process; timeline of the last step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/tools/ab_inproc.py --score rank --rounds 1 --steps 2 base: > $O/tr.log 2>&1 || { tail -20 $O/tr.log; exit 1; }
F=$(find $O/tr -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline.py $F > $O/rank_timeline.txt
grep -v copyBuffer $O/rank_timeline.txt | tail -60
