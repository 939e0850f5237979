#!/bin/bash
# Config 5 pipelined vs serial, alternated twice.  Usage: tools/gpu_cfg5ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for r in 1 2; do
  for m in pipe serial; do
    X=""; [ $m = serial ] && X="--genomes-serial"
    timeout -k 10 300 python bench.py --mode genomes --genomes-per-rank 4 --no-cpu $X --out $O/g4_${m}_$r.json > $O/g4_${m}_$r.log 2>&1 || { tail -20 $O/g4_${m}_$r.log; exit 1; }
    python3 -c "import json; b=json.load(open('$O/g4_${m}_$r.json')); print('$m', $r, b['value'], b['ms_per_step'])"
  done
done
