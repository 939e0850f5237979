#!/bin/bash
# GPU suite, then the in-process count A/B and config 5 (tools/gpu_count_inproc.sh).
# Usage: tools/gpu_count_ab2.sh TAG "variants..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$1
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$1/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/$1/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/$1/pytest_gpu.txt
bash tools/gpu_count_inproc.sh "$1" "$2"
