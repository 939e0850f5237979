#!/bin/bash
# Session-3: the small-grid gated second passes as a variant library
# (libkmerspans_gated.so, KS_LIB_PATH): GPU tests of the carry / fallback
# paths with it, then in-process A/B of its grid against the full grid
# (KS_GATED_FULL), then alternating bench runs against the in-tree build.
set -e
O=gpurun_out/s3j
mkdir -p $O
V=$PWD/kmer_spans_amd/libkmerspans_gated.so
KS_LIB_PATH=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gated.txt 2>&1
KS_LIB_PATH=$V timeout -k 10 300 python tools/ab_inproc.py --rounds 4 --steps 3 small: full:KS_GATED_FULL=1 > $O/ab_gated_inproc.txt 2>&1
bash tools/ab_bench.sh s3j "--steps 5 --warmup 1 --no-cpu --no-visits" base gated base gated > $O/ab_gated_bench.txt 2>&1
