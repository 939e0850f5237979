#!/bin/bash
# Which earlier GPU test file makes test_gpu_parity.py's host-entry cases
# fail: each set once, in its own process.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-bisect}
mkdir -p $O
cd $R
P=tests/test_gpu_parity.py
run() { tag=$1; shift; timeout -k 10 400 python -u -m pytest "$@" -m gpu -q --timeout 300 --timeout-method thread > $O/$tag.txt 2>&1; rc=$?; echo "$tag rc $rc $(tail -1 $O/$tag.txt)"; grep -h "^FAILED" $O/$tag.txt | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run parity $P
run guard tests/test_gpu_ctx_guard.py $P
run exact tests/test_gpu_exact.py $P
run configs_lines tests/test_gpu_configs.py tests/test_gpu_lines.py $P
run all_before tests/test_gpu_configs.py tests/test_gpu_ctx_guard.py tests/test_gpu_exact.py tests/test_gpu_lines.py $P
