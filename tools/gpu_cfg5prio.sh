#!/bin/bash
# Config 5 pipelined with the next genome's count stream at each torch priority.
# Usage: tools/gpu_cfg5prio.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 120 python -c "import torch; print('priority_range', torch.cuda.Stream.priority_range())"
for r in 1 2; do
  for P in none 0 -1 1; do
    X=""; [ $P != none ] && X="--count-priority $P"
    timeout -k 10 300 python bench.py --mode genomes --genomes-per-rank 4 --no-cpu $X --out $O/g4_p${P}_$r.json > $O/g4_p${P}_$r.log 2>&1 || { echo "FAILED $P"; tail -5 $O/g4_p${P}_$r.log; continue; }
    python3 -c "import json; b=json.load(open('$O/g4_p${P}_$r.json')); print('prio $P', $r, b['value'], b['ms_per_step'])"
  done
done
