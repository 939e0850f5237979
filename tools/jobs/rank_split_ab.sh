#!/bin/bash
# Count A/B, weighted-rank split A/B (in process), then the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
V="old:KS_SCATTER_STAGE=0 s16x1024:KS_SCATTER_STAGE=16x1024 s16x512:KS_SCATTER_STAGE=16x512"
timeout -k 10 300 python -u tools/ab_count.py --rounds 3 --steps 2 --k 13 $V > $O/ab_count_k13.txt 2>&1 || { tail -20 $O/ab_count_k13.txt; exit 1; }
tail -5 $O/ab_count_k13.txt
V="nosplit:KS_NO_F64_SPLIT=1 ser70:KS_SPLIT_FRAC=0.7 ser60:KS_SPLIT_FRAC=0.6 ser65:KS_SPLIT_FRAC=0.65 conc70:KS_F64_P1_CONC=1,KS_SPLIT_FRAC=0.7"
timeout -k 10 400 python -u tools/ab_inproc.py --score rank --rounds 3 --steps 2 $V > $O/ab_rank.txt 2>&1 || { tail -20 $O/ab_rank.txt; exit 1; }
tail -6 $O/ab_rank.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
