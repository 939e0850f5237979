#!/bin/bash
# In-process A/B: the second part's pass 1 after the first's (KS_P1_SERIAL) vs at once, by split fraction.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
V="base: ser:KS_P1_SERIAL=1 ser75:KS_P1_SERIAL=1,KS_SPLIT_FRAC=0.75 ser80:KS_P1_SERIAL=1,KS_SPLIT_FRAC=0.8 ser85:KS_P1_SERIAL=1,KS_SPLIT_FRAC=0.85"
timeout -k 10 400 python -u tools/ab_inproc.py --rounds 3 --steps 3 $V > $O/ab_genome.txt 2>&1 || { tail -20 $O/ab_genome.txt; exit 1; }
tail -12 $O/ab_genome.txt
V="base: ser:KS_P1_SERIAL=1 ser85:KS_P1_SERIAL=1,KS_SPLIT_FRAC=0.85 ser90:KS_P1_SERIAL=1,KS_SPLIT_FRAC=0.9 f70:KS_SPLIT_FRAC=0.7"
timeout -k 10 400 python -u tools/ab_inproc.py --rounds 3 --steps 3 --shard-of 8 $V > $O/ab_shard8.txt 2>&1 || { tail -20 $O/ab_shard8.txt; exit 1; }
tail -12 $O/ab_shard8.txt
