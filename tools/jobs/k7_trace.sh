#!/bin/bash
# Kernel trace of the small-k (k = 7, +-1) step; timeline of the last step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/tools/ab_inproc.py --k 7 --score pm1 --rounds 1 --steps 2 base: > $O/tr.log 2>&1 || { tail -20 $O/tr.log; exit 1; }
F=$(find $O/tr -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline.py $F > $O/k7_timeline.txt
grep -v copyBuffer $O/k7_timeline.txt | awk '$6+0 > 30' | tail -40
