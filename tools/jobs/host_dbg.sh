#!/bin/bash
# Phase times of the host entry point (ks_kmer_regions with visits) on the metric genome.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
KS_DEBUG_HOST=1 timeout -k 10 600 python bench.py --no-cpu --no-rank --no-visits --steps 2 --out $O/bench.json > $O/log.txt 2>&1 || { tail -20 $O/log.txt; exit 1; }
grep "host kmer_regions" $O/log.txt
python -c "import json;b=json.load(open('$O/bench.json'));print(b['host_path'])"
