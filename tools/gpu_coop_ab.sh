#!/bin/bash
# GPU suite, then in-process A/B of the carry's cooperative FP64 line fetch
# (weighted rank k = 13 and k = 15).  Usage: tools/gpu_coop_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 600 python tools/ab_inproc.py --score rank --k 13 --rounds 3 --steps 2 coop: lane:KS_NO_COOP=1 > $O/ab_k13.txt 2>&1 || { tail -30 $O/ab_k13.txt; exit 1; }
grep -v "^{" $O/ab_k13.txt | tail -4
