#!/bin/bash
# Count A/B (in process, counts must be equal across variants) + the GPU tests that count.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
V="old:KS_SCATTER_STAGE=0 s32x1024:KS_SCATTER_STAGE=32x1024 s32x512:KS_SCATTER_STAGE=32x512 s16x1024:KS_SCATTER_STAGE=16x1024 s16x512:KS_SCATTER_STAGE=16x512"
timeout -k 10 300 python -u tools/ab_count.py --rounds 3 --steps 2 --k 13 $V > $O/ab_k13.txt 2>&1 || { tail -20 $O/ab_k13.txt; exit 1; }
tail -7 $O/ab_k13.txt
for K in 11 12; do
timeout -k 10 200 python -u tools/ab_count.py --rounds 1 --steps 1 --k $K --scale 0.1 old:KS_SCATTER_STAGE=0 s32:KS_SCATTER_STAGE=32x1024 s16:KS_SCATTER_STAGE=16x512 > $O/ab_k$K.txt 2>&1 || { tail -20 $O/ab_k$K.txt; exit 1; }
tail -3 $O/ab_k$K.txt
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_tables.py tests/test_ingest.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
