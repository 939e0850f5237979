#!/bin/bash
# In-process A/B of scan knobs on the metric genome (tools/ab_inproc.py),
# then (optional) a kernel trace of the bench with the given environment.
# Usage: tools/gpu_ab.sh TAG "ab_inproc args..." ["ENV=V ENV=V" for the trace]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u tools/ab_inproc.py $2 --out $O/ab.json > $O/ab.txt 2>&1 || { tail -30 $O/ab.txt; exit 1; }
cat $O/ab.txt
if [ -n "$3" ]; then
  export TMPDIR=/tmp
  cd /tmp
  env $3 true
  for kv in $3; do export $kv; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-rank --no-host-path --no-visits --out $O/prof_bench.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  F=$(find $O/prof -name '*kernel_trace.csv' | head -1)
  python3 $R/tools/timeline.py $F > $O/step_timeline.txt || true
  grep -E "k_pass1|k_p1_gate|k_stitch_emit|k_scan_lane|k_copy_u64" $O/step_timeline.txt | tail -12
fi
