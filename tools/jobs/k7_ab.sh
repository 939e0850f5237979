#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallk.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_smallk.txt 2>&1 || { tail -30 $O/pytest_smallk.txt; exit 1; }
tail -1 $O/pytest_smallk.txt
timeout -k 10 400 python -u tools/ab_inproc.py --k 7 --score pm1 --rounds 3 --steps 2 base: glob:KS_SUMM_GLOBAL_TAB=1 > $O/ab_k7_pm1.txt 2>&1 || { tail -20 $O/ab_k7_pm1.txt; exit 1; }
tail -3 $O/ab_k7_pm1.txt
timeout -k 10 400 python -u tools/ab_inproc.py --k 7 --score log2 --rounds 3 --steps 2 base: glob:KS_SUMM_GLOBAL_TAB=1 > $O/ab_k7_log2.txt 2>&1 || { tail -20 $O/ab_k7_log2.txt; exit 1; }
tail -3 $O/ab_k7_log2.txt
