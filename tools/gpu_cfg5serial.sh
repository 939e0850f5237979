#!/bin/bash
# Config 5 serial genomes: one genome's phases and a kernel trace (timeline)
# of the serial bench line.  Usage: tools/gpu_cfg5serial.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python tools/genome_phases.py --ext-gib 32 --reps 2 > $O/phases_32.txt 2>&1 || { tail -20 $O/phases_32.txt; exit 1; }
tail -3 $O/phases_32.txt
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --mode genomes --genomes-per-rank 3 --genomes-serial --no-cpu --out $O/g3.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
F=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline.py $F > $O/timeline.txt || true
find $O/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} sh -c 'cut -c1-150 {} | head -30'
