#!/bin/bash
# Kernel timeline of one scan step.  Usage: tools/jobs/shard_tl.sh TAG [S] [bench args...]
# (S = --shard-of: the step of the largest of S LPT shards)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
S=${2:-8}
shift; shift
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python $R/bench.py --shard-of $S \
  --steps 2 --warmup 1 --no-cpu --no-rank --no-host-path --no-visits "$@" > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
F=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python $R/tools/timeline.py $F > $O/timeline.txt && grep -v rocclr_copyBuffer $O/timeline.txt | awk '$6 > 30 || /span/'
