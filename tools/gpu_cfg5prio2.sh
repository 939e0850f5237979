#!/bin/bash
# Config 5 pipelined: default count stream vs high priority, alternated 3 times.
# Usage: tools/gpu_cfg5prio2.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for r in 1 2 3; do
  for P in none -1; do
    X=""; [ $P != none ] && X="--count-priority $P"
    timeout -k 10 300 python bench.py --mode genomes --genomes-per-rank 4 --no-cpu $X --out $O/g4_p${P}_$r.json > $O/g4_p${P}_$r.log 2>&1 || { echo "FAILED $P"; tail -5 $O/g4_p${P}_$r.log; exit 1; }
    python3 -c "import json; b=json.load(open('$O/g4_p${P}_$r.json')); print('prio $P', $r, b['value'], b['ms_per_step'])"
  done
done
