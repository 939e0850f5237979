#!/bin/bash
# GPU suite, the k = 13 count in one process, and the config-5 phase breakdown.
# Usage: tools/gpu_count_ab.sh TAG
set -o pipefail
mkdir -p gpurun_out/${1:-count}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${1:-count}/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/${1:-count}/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/${1:-count}/pytest_gpu.txt
timeout -k 10 300 python tools/ab_count.py --k 13 --rounds 2 new: > gpurun_out/${1:-count}/count.txt 2>&1 || { tail -20 gpurun_out/${1:-count}/count.txt; exit 1; }
cat gpurun_out/${1:-count}/count.txt
bash tools/gpu_cfg5prof.sh ${1:-count}
