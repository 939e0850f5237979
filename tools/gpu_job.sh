#!/bin/bash
# scratch GPU job of the current session (see the commands below)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-job}
mkdir -p $O
cd $R
V="one:KS_PARTS_FRAC=0 p55:KS_PARTS_FRAC=0.55 p65:KS_PARTS_FRAC=0.65 p75:KS_PARTS_FRAC=0.75 p55h:KS_PARTS_FRAC=0.55,KS_PARTS_HALVES=1"
timeout -k 10 600 python -u tools/ab_inproc.py --rounds 3 --steps 3 $V --out $O/ab_log2.json > $O/ab_log2.txt 2>&1 || { tail -30 $O/ab_log2.txt; exit 1; }
tail -6 $O/ab_log2.txt
timeout -k 10 600 python -u tools/ab_inproc.py --rounds 3 --steps 3 --shard-of 8 $V --out $O/ab_shard8.json > $O/ab_shard8.txt 2>&1 || { tail -30 $O/ab_shard8.txt; exit 1; }
tail -6 $O/ab_shard8.txt
timeout -k 10 900 python -u tools/ab_inproc.py --rounds 3 --steps 2 --score rank $V --out $O/ab_rank.json > $O/ab_rank.txt 2>&1 || { tail -30 $O/ab_rank.txt; exit 1; }
tail -6 $O/ab_rank.txt
