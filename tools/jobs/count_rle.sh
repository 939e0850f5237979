#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "hot_buckets or chr1" -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash tools/jobs/bins_ab.sh $1
