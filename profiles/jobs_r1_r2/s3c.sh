#!/bin/bash
# Session-3: visit-histogram mode tests, expanded-table build A/B (4 pairs per
# lane and trip vs 1), split fraction re-check after the faster run pass.
set -e
O=gpurun_out/s3c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "visit_histogram or human_like or expanded" > $O/pytest_visits.txt 2>&1
timeout -k 10 300 python tools/ab_table.py --rounds 4 u4: u1:KS_EXT_U1=1 > $O/ab_table.txt 2>&1
timeout -k 10 300 python tools/ab_inproc.py --rounds 4 --steps 3 f70: f65:KS_SPLIT_FRAC=0.65 f75:KS_SPLIT_FRAC=0.75 > $O/ab_split.txt 2>&1
