#!/bin/bash
# New count test, then the per-config bench lines.  Usage: tools/jobs/cfg_test.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k hot_buckets -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_hot.txt 2>&1 || { tail -30 $O/pytest_hot.txt; exit 1; }
tail -1 $O/pytest_hot.txt
bash tools/jobs/configs.sh $1
