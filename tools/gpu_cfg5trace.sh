#!/bin/bash
# Kernel trace (timeline) of the pipelined config-5 line.  Usage: tools/gpu_cfg5trace.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --mode genomes --genomes-per-rank 3 --no-cpu --out $O/g3.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
F=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline.py $F > $O/timeline.txt || true
wc -l $O/timeline.txt
