#!/bin/bash
# rocprofv3 kernel stats of the metric step, line tables vs the expanded table.  Usage: tools/jobs/prof_ab.sh TAG
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in lines ext; do
  if [ $v = ext ]; then export KS_NO_LINES=1; else unset KS_NO_LINES; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-visits --no-rank --no-host-path > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  f=$(find $O/prof_$v -name '*kernel_stats.csv' | head -1)
  head -25 $f | cut -d, -f1-6
  t=$(find $O/prof_$v -name '*kernel_trace.csv' | head -1)
  python3 $R/tools/timeline.py $t > $O/timeline_$v.txt 2>&1 || true
done
