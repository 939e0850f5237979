#!/bin/bash
# Kernel trace of the weighted-rank (config 3) step with the given environment
# (one step after a warm-up), and its step timeline.  Usage: tools/gpu_rankprof2.sh TAG "ENV=V ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
for kv in $2; do export $kv; done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --score rank --steps 2 --warmup 1 --no-cpu --no-rank --no-host-path --no-visits --out $O/bench.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
F=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline.py $F > $O/step_timeline.txt || true
tail -60 $O/step_timeline.txt
