#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4m
mkdir -p $O
cd $R
B="timeout -k 10 400 python -u bench.py --mode genomes --genomes-per-rank 4 --no-cpu"
$B --out $O/g_q4.json > $O/g_q4.log 2>&1 || { tail -20 $O/g_q4.log; exit 1; }
GPU_MAX_HW_QUEUES=8 $B --out $O/g_q8.json > $O/g_q8.log 2>&1 || { tail -20 $O/g_q8.log; exit 1; }
GPU_MAX_HW_QUEUES=16 $B --out $O/g_q16.json > $O/g_q16.log 2>&1 || { tail -20 $O/g_q16.log; exit 1; }
M="timeout -k 10 300 python -u bench.py --no-cpu --no-rank --no-host-path --no-visits --steps 10"
$M --out $O/m_q4.json > $O/m_q4.log 2>&1 || { tail -20 $O/m_q4.log; exit 1; }
GPU_MAX_HW_QUEUES=8 $M --out $O/m_q8.json > $O/m_q8.log 2>&1 || { tail -20 $O/m_q8.log; exit 1; }
$M --out $O/m_q4b.json > $O/m_q4b.log 2>&1 || { tail -20 $O/m_q4b.log; exit 1; }
for f in g_q4 g_q8 g_q16 m_q4 m_q8 m_q4b; do python3 -c "import json;b=json.load(open('$O/$f.json'));print('$f', b['value'], b['ms_per_step'])"; done
