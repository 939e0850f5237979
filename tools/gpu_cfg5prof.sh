#!/bin/bash
# Config 5 (genomes per GPU) phase breakdown: one genome's count / table / scan
# at several expansion caps, and a kernel trace of the pipelined bench line.
# Usage: tools/gpu_cfg5prof.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for g in 16 32 64; do
  timeout -k 10 300 python tools/genome_phases.py --ext-gib $g --reps 2 > $O/phases_$g.txt 2>&1 || { tail -20 $O/phases_$g.txt; exit 1; }
  tail -1 $O/phases_$g.txt
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --mode genomes --genomes-per-rank 3 --no-cpu --out $O/g3.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
F=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline.py $F > $O/timeline.txt || true
find $O/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} sh -c 'cut -c1-150 {} | head -30'
