#!/bin/bash
# In-process count A/B (tools/ab_count.py variants) and config 5 serial vs pipelined.
# Usage: tools/gpu_count_inproc.sh TAG "variants..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python tools/ab_count.py --k 13 --rounds 3 $2 > $O/count_ab.txt 2>&1 || { tail -20 $O/count_ab.txt; exit 1; }
cat $O/count_ab.txt
timeout -k 10 600 python bench.py --mode genomes --genomes-per-rank 4 --no-cpu --out $O/g4_pipe.json > $O/g4_pipe.log 2>&1 || { tail -20 $O/g4_pipe.log; exit 1; }
timeout -k 10 600 python bench.py --mode genomes --genomes-per-rank 4 --no-cpu --genomes-serial --out $O/g4_serial.json > $O/g4_serial.log 2>&1 || { tail -20 $O/g4_serial.log; exit 1; }
python3 -c "import json
for t in ('pipe','serial'):
    b=json.load(open('$O/g4_'+t+'.json')); print(t, b['value'], b['ms_per_step'])"
